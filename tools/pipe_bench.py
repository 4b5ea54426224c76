"""Config 3 only (bench.py's single_stream leg, no CPU oracle): the sequential node chain and the
node pipeline, with each pipeline node's busy time per sweep.  Prints one JSON line."""
import importlib
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402

loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
if os.environ.get("PIPE_SWITCH"):
    sys.setswitchinterval(float(os.environ["PIPE_SWITCH"]))
print(json.dumps(bench.stream_leg(loam, sg, int(os.environ.get("STREAM_SWEEPS", "220")), 0,
                                  stages=int(os.environ.get("PIPE_STAGES", "3")),
                                  priority=json.loads(os.environ["PIPE_PRIO"]) if "PIPE_PRIO" in os.environ else "default")))
