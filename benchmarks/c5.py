"""C5: the skewed 2-relation join (BASELINE.json configs[4]) -- §8(f) row f-2.

Workload: qe.datagen.c5_spec(N): r0 = (v % N, Zipf key, u32), r1 = (Zipf key, v % N, u32) with
N = 1e9 rows per side, Zipf(0.9) over D = N through one shared rank->key permutation, generated
in HBM (libqe builds the Zipf CDF on the device in a fixed summation order, so every run draws
the same keys, and samples it with its kind-2 generator).  Query `0 1|0.1=1.0|0.2 1.2`.

The join has P ~ 3.8e14 pairs: no machine materialises that, and the reference's DArray caps a
list at INT32_MAX elements (src/DArray.h:14-15).  libqe's executor therefore takes the aggregate
form of the merge (qe_merge_join_counts: each row's partner count on both sides) and prints
sum_i col[rowid_i] * count_i per select, which is exactly the checksum of the list the
reference would build (proved against the reference at 20 k rows in §9.5 and
checked here against the C5 goldens and against numpy aggregate truth at 1e8 rows).
One step = one execution of the query (both sorts, both count passes, both checksums).
`value` = input rows (both sides) per second; the join's pair count (counted, not materialised)
is reported beside it as `pairs` and `pairs_counted_per_s`.
"""
from __future__ import annotations

import os
import time

from qe import datagen as dg

from .cpuref import CpuRef, cpu_model, pin_one_core

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METRIC = "input rows/sec, C5 2-relation Zipf(0.9) join, 1e9 rows/side (pairs counted, not materialised)"


gen_c5 = dg.gen_c5

PATH_ONE_RANK = ("qe_run_queries_dist on one rank (the product default): the plan's last join of two base "
                 "relations in aggregate form (engine join_agg, csrc/qe_comm.hip e_join_agg -> qe_join_aggregate, "
                 "csrc/qe_agg.hip): per side a histogram read and the two-level sort's two lookback-free "
                 "partition passes of (key field << 32 | select value) words into 2^15 buckets "
                 "(partition_words_kv), then one counting workgroup per bucket (ab_bucket_kernel: S's key "
                 "counts in LDS, R rows add pairs and valR*cnt, then R's counts, S rows add valS*cnt; head keys "
                 "beyond 2^18 rows per bucket side on the chunked giant path)")
PATH_N_RANKS = ("qe_run_queries_dist (host-C plan, include/qe_plan.h) over RCCL: e_join_agg at N ranks -- heavy "
                "keys (sampled from the replicated key columns) counted over each rank's row slice and "
                "all-reduced, light keys hash-bucketed locally from the replicated columns (bucket_select_dev) "
                "and joined by the bucketed aggregate join above; sums all-reduced")


# what `parity` means at 1e9 rows: self-consistency, not a reference output -- the reference
# binary cannot run this size; the constants are an independent aggregate (torch, key-range sharded)
# over the same device columns, and that aggregate is pinned to the reference's own G1-G3 outputs on CPU
# (tests/test_agg_truth.py); the C5 goldens (tests/golden/c5*.json) are the reference-pinned cases
PARITY_BASIS = ("self-consistency at 1e9 rows (parity unpinned vs the reference binary at this size): equal to "
                "an independent key-range-sharded aggregate over the same columns, itself pinned to the "
                "reference's G1-G3 outputs; the reference-pinned C5 cases are tests/golden/c5*.json")


def pinned_parity(rows: int, out: str, pairs: int):
    """the line against the pinned 1e9 output (qe.datagen.C5_1E9_*); None at other sizes"""
    if rows != dg.C5_ROWS:
        return None
    return out == dg.C5_1E9_STDOUT and pairs == dg.C5_1E9_PAIRS


def cpu_sample(ctx, sample_rows: int, budget_note: str = "") -> dict:
    """oracle/cpu_ref, one core, on the first `sample_rows` rows of both relations (same Zipf
    columns, so the heavy keys collide as at full size; the join is small enough to
    materialise).  The GPU runs the same sample through both of its paths for a byte check."""
    from qe import lib
    cols = [[ctx.column_range_to_host(r, c, 0, sample_rows) for c in range(3)] for r in range(2)]
    cr = CpuRef()
    for cs in cols:
        cr.add_relation(cs)
    pin_one_core()
    cpu_out, _, dt = cr.run(dg.C5_QUERY)
    cr.close()
    # the same sample on the GPU: materialised (default limit) and aggregate (limit 0)
    g = lib.Ctx(ctx.device) if hasattr(ctx, "device") else lib.Ctx(0)
    for cs in cols:
        g.load_relation(cs)
    mat, _ = g.run(dg.C5_QUERY)
    pairs = g.last_result_rows()
    g.set_materialize_limit(0)
    agg, _ = g.run(dg.C5_QUERY)
    g.close()
    return {"value": round(2 * sample_rows / dt, 1), "unit": "input rows/s", "cores": 1, "kind": "port",
            "sample": f"first {sample_rows} rows of both C5 relations (same device-made Zipf columns), "
                      f"{pairs} pairs materialised by oracle/cpu_ref single-threaded in {dt:.2f} s{budget_note}",
            "seconds": round(dt, 3), "pairs": pairs,
            "pairs_per_s": round(pairs / dt, 1), "cpu_model": cpu_model(),
            "parity_with_gpu": cpu_out == mat == agg}


def run_single(args, log, roofline_fn=None, traffic_fn=None) -> dict:
    import torch

    from qe import lib
    torch.cuda.init()
    rows = args.rows or dg.C5_ROWS
    ctx = lib.Ctx(0)
    t0 = time.time()
    gen_c5(ctx, rows)
    log(f"[c5] 2 x {rows} rows (Zipf {dg.C5_THETA}) in HBM in {time.time() - t0:.1f}s")
    out = None
    for _ in range(args.warmup):
        out, rc, _ = ctx.run_dist(dg.C5_QUERY)
    ctx.set_profiling(True)
    ctx.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, rc, refused = ctx.run_dist(dg.C5_QUERY)
    ctx.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pairs = ctx.last_result_rows()
    stats = ctx.kernel_stats()
    ctx.set_profiling(False)
    kern = sorted(stats.items(), key=lambda kv: -kv[1]["ms"])
    ms = dt / args.steps * 1e3
    res = {
        "metric": METRIC, "value": round(2 * rows * args.steps / dt, 1), "unit": "input rows/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: qe.datagen.c5_spec(%d) generated in HBM (seed %d, Zipf %.1f, shared permutation)"
                % (rows, dg.C5_SEED, dg.C5_THETA),
        "parity": pinned_parity(rows, out, pairs),
        "parity_basis": PARITY_BASIS,
        "parity_detail": {"equals_pinned_c5_1e9": pinned_parity(rows, out, pairs),
                          "pinned_by": "tests/test_gpu_fullsize_batch.py (sharded aggregate truth on the device columns)"},
        "config": {"workload": "C5: 2-relation join, %d rows/side, Zipf theta=%.1f keys, query %s"
                               % (rows, dg.C5_THETA, dg.C5_QUERY.strip()),
                   "pairs": pairs, "materialised": False,
                   "path": PATH_ONE_RANK, "refused": refused,
                   "pairs_counted_per_s": round(pairs * args.steps / dt, 1),
                   "stdout": out, "parallelism": "single GPU"},
        "roofline": roofline_fn(stats, traffic_fn() if traffic_fn else None) if roofline_fn else None,
        "stages": {k: {"ms_per_step": round(s["ms"] / args.steps, 3), "launches_per_step": s["launches"] / args.steps}
                   for k, s in kern[:10]},
    }
    if not args.no_cpu:
        res["cpu_baseline"] = cpu_sample(ctx, args.cpu_rows_c5)
    else:
        res["cpu_baseline"] = None
    ctx.close()
    return res


def run_dist(args, log) -> dict | None:
    """C5 on N ranks (one per GPU): qe_run_queries_dist over an RCCL communicator (gloo carries only
    the bootstrap id, the barriers and the max time).  The C plan runs the query's one join -- its
    last, of two whole base relations -- in the engine's aggregate form: heavy keys (sampled from the
    replicated key columns) counted per row slice and all-reduced, light keys hash-bucketed locally
    from the replicated columns and joined in aggregate form, sums all-reduced.  Strong scaling:
    `--rows` (default 1e9) rows per side in total."""
    import torch
    import torch.distributed as dist

    from qe import lib
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    torch.cuda.init()
    solo = world == 1
    if not solo and not dist.is_initialized():
        dist.init_process_group("gloo")
    rows = args.rows or dg.C5_ROWS
    ctx = lib.Ctx(dev)
    comm = None
    if not solo:
        box = [lib.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        comm = lib.Comm(ctx, world, rank, box[0])   # the data path: RCCL over xGMI
    t0 = time.time()
    gen_c5(ctx, rows)
    ctx.sync()
    if rank == 0:
        log(f"[c5] {world} rank(s): 2 x {rows} rows (Zipf {dg.C5_THETA}) replicated in HBM in {time.time() - t0:.1f}s")
    q = dg.C5_QUERY
    out = None
    for _ in range(args.warmup):
        out, rc, refused = ctx.run_dist(q, comm)
    ctx.set_profiling(True)
    ctx.reset_stats()
    if not solo:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, rc, refused = ctx.run_dist(q, comm)
    ctx.sync()
    torch.cuda.synchronize()
    if not solo:
        dist.barrier()
    dt = time.perf_counter() - t0
    if not solo:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    pairs = ctx.last_result_rows()
    stats = ctx.kernel_stats()
    ctx.set_profiling(False)
    res = None
    if rank == 0:
        kern = sorted(stats.items(), key=lambda kv: -kv[1]["ms"])
        res = {
            "metric": METRIC, "value": round(2 * rows * args.steps / dt, 1), "unit": "input rows/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic: qe.datagen.c5_spec(%d) generated in HBM on every rank (seed %d, Zipf %.1f)"
                    % (rows, dg.C5_SEED, dg.C5_THETA),
            "parity": pinned_parity(rows, out, pairs),
            "parity_basis": PARITY_BASIS,
            "config": {"workload": "C5: 2-relation join, %d rows/side in total, Zipf theta=%.1f keys, query %s"
                                   % (rows, dg.C5_THETA, q.strip()),
                       "pairs": pairs, "materialised": False, "refused": refused,
                       "path": PATH_N_RANKS if world > 1 else PATH_ONE_RANK,
                       "pairs_counted_per_s": round(pairs * args.steps / dt, 1),
                       "stdout": out,
                       "parallelism": f"hash buckets + heavy split x{world}" if world > 1 else "single GPU"},
            "stages": {k: {"ms_per_step": round(s["ms"] / args.steps, 3)} for k, s in kern[:10]},
            "cpu_baseline": None,
        }
    if comm is not None:
        comm.close()
    if not solo:
        dist.barrier()
    ctx.close()
    if not solo:
        dist.destroy_process_group()
    return res
