"""The oracle against its committed regression vectors (tests/golden/oracle_golden.json, made by
tests/golden/make_golden.py).  Parity with the reference itself is unpinned."""
import hashlib
import json
import os

import numpy as np

G = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_golden.json")))


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def test_config2_scan_registration(oc, sg):
    prev, cur = sg.single_problem(0)
    o = oc.Oracle(oc.default_config(system_delay=1))
    o.scan_registration(cur)
    rc, f = o.scan_registration(cur)
    for k, v in G["config2_sr_cur"].items():
        assert f[k].shape[0] == v["count"], k
        assert digest(f[k]) == v["sha256"], k


def test_config2_problem(oc, sg):
    prev, cur = sg.single_problem(0)
    od, aft, st = oc.problem(prev, cur)
    np.testing.assert_array_equal(od, np.float32(G["config2_problem"]["od_sum"]))
    np.testing.assert_array_equal(aft, np.float32(G["config2_problem"]["aft"]))


def test_config4_first8(oc, sg):
    prevs, curs = sg.batch_problems(8, base_seed=1000)
    for i in range(8):
        od, aft, _ = oc.problem(prevs[i], curs[i])
        np.testing.assert_array_equal(od, np.float32(G["config4_first8"][i]["od_sum"]))
        np.testing.assert_array_equal(aft, np.float32(G["config4_first8"][i]["aft"]))
