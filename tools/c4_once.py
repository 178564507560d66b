"""One C4 batch on the lanes, bracketed by CLOCK_MONOTONIC stamps (for a rocprofv3 kernel-trace timeline):
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/c4_once.py STAMPFILE [plan|faithful] [workers]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-compiler-executor_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from benchmarks import c4  # noqa: E402
from qe import datagen as dg  # noqa: E402
from qe import lib  # noqa: E402

stamp = sys.argv[1]
plan = (sys.argv[2] if len(sys.argv) > 2 else "plan") == "plan"
workers = int(sys.argv[3]) if len(sys.argv) > 3 else 8
torch.cuda.init()
c4.install_crash_maps()
ctx = lib.Ctx(0)
queries = c4.load_queries()
text = dg.c4_batches(queries)
c4.gen_c4(ctx)
ctx.run_lanes(text, workers, plan=plan)
ctx.sync()
t0 = time.monotonic_ns()
out, rc = ctx.run_lanes(text, workers, plan=plan)
ctx.sync()
t1 = time.monotonic_ns()
with open(stamp, "w") as f:
    f.write(f"{t0} {t1}\n")
print(f"batch {(t1 - t0) / 1e6:.1f} ms rc {rc} lines {out.count(chr(10))}")
ctx.close()
