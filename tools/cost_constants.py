"""Per-row costs behind the partitioned plan's broadcast-or-partition choice (host/qe_plan.c
bcast_join), measured on this GPU:  python3 tools/cost_constants.py > profiles/TAG_cost_constants.json

* partition: qe_partition (partition_dev: count + stable scatter) of a C3-sized derived side --
  46.6 M rows, u64 keys < 1e8 and two u32 columns -- into 2 / 4 / 8 destinations; ps per row
  (the plan's exchange sends u32 keys, so this 8-B-key figure is an upper bound);
* bucket select: qe_bucket_select of a 1e8-row base column (the lazily built base bucket, paid once
  per column and rank count);
The sort and bucket-join per-row figures come from the same run's C3 kernel trace
(tools/trace_launches.py), not from here."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-compiler-executor_amd"))

import torch  # noqa: E402

from qe import lib  # noqa: E402


def timed(f, reps=10, warm=2):
    for _ in range(warm):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    torch.cuda.init()
    ctx = lib.Ctx(0)
    n = 46_600_000
    g = torch.Generator(device="cuda").manual_seed(1)
    keys = torch.randint(0, 100_000_000, (n,), dtype=torch.int64, device="cuda", generator=g)
    cols = [torch.randint(0, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g) for _ in range(2)]
    ok = torch.empty_like(keys)
    oc = [torch.empty_like(c) for c in cols]
    res = {"rows": n, "partition_ps_per_row": {}, "note": "u64 keys in and out, 2 u32 columns (C3's J1 shape)"}
    for G in (2, 4, 8):
        dt = timed(lambda: ctx.partition(keys.data_ptr(), n, [c.data_ptr() for c in cols], G, ok.data_ptr(),
                                         [o.data_ptr() for o in oc]))
        res["partition_ps_per_row"][G] = round(dt / n * 1e12, 2)
    N = 100_000_000
    ctx.gen_relation(N, [("mod", N), ("mod", N), ("hi32",)], seed=1, gen_rel=0)
    col = ctx.column(0, 1)
    res["bucket_select_ps_per_row"] = {}
    for G in (2, 8):
        def sel():
            p = ctx.bucket_select(col, G, 0)
            ctx.pairs_free(p)
        res["bucket_select_ps_per_row"][G] = round(timed(sel, reps=5) / N * 1e12, 2)
    res["device"] = ctx.device_name()
    ctx.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
