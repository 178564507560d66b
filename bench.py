#!/usr/bin/env python3
"""bench.py -- the headline benchmark: joined tuples/s on the 4-relation chain join (config C3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--no-cpu] [--workload c3|c4|c5]

Workload (BASELINE.json configs[2]): four relations of R = 100 M rows
(c0 = v % R, c1 = v % R, c2 = v >> 32, splitmix64 seed 1, generated straight into HBM), query
    0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2
One step = one full execution of that query: both filters, three sort-merge joins, the
mid_result payload propagation and the three checksums, printed exactly as the reference
prints them.  `value` = chain rows produced per second (joined tuples/s), whole job.

N = 1 runs libqe's faithful executor (the drop-in for the reference's execute_query).  N > 1
runs the key-partitioned plan of qe.dist: every rank owns R rows of every
relation (weak scaling), rows are hash-partitioned on the join key and exchanged with an RCCL
all-to-all per join, and the checksums are all-reduced.

The JSON line also carries `roofline` (the dominant kernel's algorithmic GB/s from HIP events on
the libqe stream, against the 8 TB/s HBM3E peak) and `cpu_baseline` (oracle/cpu_ref, the C
restatement of the reference path, single-threaded on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "query-compiler-executor_amd"))
sys.path.insert(0, ROOT)

METRIC = "joined tuples/sec + achieved HBM GB/s, 4-rel chain join, 1/2/4/8 MI355X"
QUERY = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_chain(ctx, rows: int, seed: int, key_domain: int, row_start: int = 0):
    kinds = [("mod", key_domain), ("mod", key_domain), ("hi32",)]
    return [ctx.gen_relation(rows, kinds, seed=seed, gen_rel=r, row_start=row_start) for r in range(4)]


def roofline(stats: dict, traffic: dict | None):
    if not stats:
        return None
    name, s = max(stats.items(), key=lambda kv: kv[1]["ms"])
    per_launch_ms = s["ms"] / max(1, s["launches"])
    per_launch_bytes = s["alg_bytes"] / max(1, s["launches"])
    achieved = per_launch_bytes / (per_launch_ms * 1e-3) / 1e9 if per_launch_ms > 0 else 0.0
    t = None
    if traffic and name in traffic:
        t = traffic[name]
    return {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": t,
            "alg_bytes_per_launch": per_launch_bytes, "avg_launch_ms": round(per_launch_ms, 4),
            "launches": s["launches"]}


def load_traffic(workload: str = "c3"):
    """HBM bytes per launch from the rocprofv3 PMC passes committed under profiles/ for this
    workload (files without a "workload" key are C3), or None -- never another workload's."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("workload", "c3") != workload:
            continue
        return {k: v.get("hbm_bytes_per_launch") for k, v in d.get("kernels", {}).items()}
    return None


def cpu_baseline(sample_rows: int, seed: int, gpu_ctx):
    """oracle/cpu_ref (single thread) on a bounded sample of the same workload; the GPU runs
    the same sample so the two outputs are compared bit for bit."""
    import ctypes as C

    import numpy as np

    from qe import datagen as dg
    so = os.path.join(ROOT, "oracle", "build", "libcpuref.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "cpuref"], check=True)
    lib = C.CDLL(so)
    lib.cpuref_create.restype = C.c_void_p
    lib.cpuref_add_relation.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p)]
    lib.cpuref_run_str.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    lib.cpuref_destroy.argtypes = [C.c_void_p]
    rels = dg.make_relations(dg.chain_spec(4, sample_rows), seed)
    h = lib.cpuref_create()
    keep = []
    for cols in rels:
        arr = (C.c_void_p * 3)(*[c.ctypes.data for c in cols])
        keep.append(arr)
        lib.cpuref_add_relation(h, sample_rows, 3, arr)
    out, n = C.c_void_p(), C.c_size_t()
    try:
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})   # one pinned core
    except Exception:
        pass
    t0 = time.perf_counter()
    rc = lib.cpuref_run_str(h, QUERY.encode(), C.byref(out), C.byref(n))
    dt = time.perf_counter() - t0
    cpu_out = C.string_at(out, n.value).decode()
    lib.cpuref_destroy(h)
    # same sample on the GPU, for a bit-exact comparison
    gpu_ctx.drop_relations()
    gen_chain(gpu_ctx, sample_rows, seed, sample_rows)
    gpu_out, _ = gpu_ctx.run(QUERY)
    rows = gpu_ctx.last_result_rows()
    gpu_ctx.drop_relations()
    del rels
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"value": round(rows / dt, 1), "unit": "joined tuples/s", "cores": 1, "kind": "port",
            "sample": f"C3 shape at {sample_rows} rows/rel (seed {seed}); oracle/cpu_ref single-threaded, "
                      f"{dt:.2f} s for {rows} chain rows",
            "seconds": round(dt, 3), "cpu_model": cpu_model, "nproc": os.cpu_count(),
            "parity_with_gpu": cpu_out == gpu_out and rc == 0, "sample_stdout": cpu_out}


def run_single(args):
    import torch

    from qe import lib
    torch.cuda.init()
    ctx = lib.Ctx(0)
    log(f"[bench] device {ctx.device_name()}")
    t0 = time.time()
    gen_chain(ctx, args.rows, args.seed, args.rows)
    ctx.sync()
    log(f"[bench] generated 4 x {args.rows} rows x 3 cols in HBM in {time.time() - t0:.2f}s")
    out = None
    for i in range(args.warmup):
        out, _ = ctx.run(QUERY)
        log(f"[bench] warmup {i}: {out.strip()!r}")
    ctx.set_profiling(True)
    ctx.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, rc = ctx.run(QUERY)
    ctx.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stats = ctx.kernel_stats()
    ctx.set_profiling(False)
    rows = ctx.last_result_rows()
    ms = dt / args.steps * 1e3
    value = rows * args.steps / dt
    # the same query with every intermediate rowid list materialised (QE_DLE=0), for the record
    dle_env = os.environ.get("QE_DLE")
    os.environ["QE_DLE"] = "0"
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        out_all, _ = ctx.run(QUERY)
    ctx.sync()
    torch.cuda.synchronize()
    dt_all = time.perf_counter() - t1
    if dle_env is None:
        del os.environ["QE_DLE"]
    else:
        os.environ["QE_DLE"] = dle_env
    kern = sorted(stats.items(), key=lambda kv: -kv[1]["ms"])
    total_kernel_ms = sum(s["ms"] for _, s in kern) / args.steps
    res = {
        "metric": METRIC, "value": round(value, 1), "unit": "joined tuples/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: splitmix64 relations generated in HBM (SURVEY.md §9.1), seed %d" % args.seed,
        "config": {"workload": "C3: 4-relation chain join R0-R1-R2-R3, 2 filters on R3, %d rows/rel" % args.rows,
                   "query": QUERY.strip(), "rows_per_relation": args.rows, "result_rows": rows,
                   "stdout": out, "executor": "libqe faithful state machine (qe_run_queries)",
                   "dead_list_elimination": os.environ.get("QE_DLE", "1") != "0",
                   "parallelism": "single GPU"},
        "all_lists_materialised": {"ms_per_step": round(dt_all / args.steps * 1e3, 3),
                                   "value": round(rows * args.steps / dt_all, 1),
                                   "stdout_identical": out_all == out},
        "roofline": roofline(stats, load_traffic()),
        "kernel_ms_per_step": round(total_kernel_ms, 3),
        "stages": {k: {"ms_per_step": round(s["ms"] / args.steps, 3), "launches_per_step": s["launches"] / args.steps,
                       "GBps": round(s["alg_bytes"] / (s["ms"] * 1e-3) / 1e9, 1) if s["ms"] > 0 else None}
                   for k, s in kern[:12]},
    }
    if not args.no_cpu:
        ctx.drop_relations()
        res["cpu_baseline"] = cpu_baseline(args.cpu_rows, args.seed, ctx)
    else:
        res["cpu_baseline"] = None
    ctx.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=None,
                    help="rows per relation (per rank for N > 1); default 1e8 (c3) / 1e9 (c5)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-rows", type=int, default=16_000_000)
    ap.add_argument("--cpu-rows-c5", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workload", choices=["c3", "c4", "c5"], default="c3",
                    help="c3 (default): the headline 4-relation chain join; c4: the SIGMOD-style batch; "
                         "c5: the skewed (Zipf 0.9) 2-relation join at 1e9 rows")
    ap.add_argument("--plan", choices=["auto", "dist"], default="auto",
                    help="auto = faithful executor at N = 1, the partitioned plan (qe.dist) at N > 1; "
                         "dist = the partitioned plan at every N (its per-rank cost at N = 1); c3 and c5")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.rows is None and args.workload != "c5":
        args.rows = 100_000_000
    if args.workload == "c5":
        from benchmarks import c5 as c5bench
        if world > 1 or args.plan == "dist":
            res = c5bench.run_dist(args, log)
        else:
            res = c5bench.run_single(args, log, roofline_fn=roofline, traffic_fn=lambda: load_traffic("c5"))
    elif args.workload == "c4":
        from benchmarks import c4 as c4bench
        if world > 1:
            res = c4bench.run_dist(args, log)
        else:
            res = c4bench.run_single(args, log, roofline_fn=roofline, traffic_fn=lambda: load_traffic("c4"))
    elif world > 1 or args.gpus > 1 or args.plan == "dist":
        from qe import dist
        res = dist.bench_main(args, METRIC, QUERY, cpu_baseline_fn=cpu_baseline, roofline_fn=roofline,
                              traffic_fn=None)
    else:
        res = run_single(args)
    if res is not None:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
