"""Phase breakdown of k_od_lm (diagnostic build: tools/build_variant.sh phases -DLOAM_PHASES):
per iteration of one workgroup, us: coefficient pass, stored-row pass, reduction, step."""
import ctypes, importlib, json, os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
prevs, curs = sg.batch_problems(B, base_seed=1000)
e = loam.Engine(device=0)
e.batch_upload(prevs, curs)
lib = ctypes.CDLL(os.environ["LOAM_HIP_LIB"])
buf = (ctypes.c_ulonglong * 27)()
e.batch_run(); e.sync()
lib.loam_debug_phases_od(buf)
a0 = list(buf)
for _ in range(3):
    e.batch_run()
e.sync()
lib.loam_debug_phases_od(buf)
a = [x - y for x, y in zip(buf, a0)]
s = a[3 + 12:3 + 24]
n = max(s[6], 1)
print(json.dumps({"batch": B, "wg_iterations": s[6], "mean_iter_index": s[4] / n,
                  "coeff_us": s[0] / n / 100, "rows_us": s[1] / n / 100, "reduce_us": s[2] / n / 100,
                  "step_us": s[3] / n / 100}))
