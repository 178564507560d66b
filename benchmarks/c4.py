"""C4: the SIGMOD-2018-style batch (BASELINE.json configs[3]) -- §8(f) row f-1.

Workload: the 14 relations of qe.datagen.c4_spec(1.0) (1e5..1e7 rows, 2..6 columns, seed 4)
generated in HBM, and the C4 queries that pass the reference's rand-invariance gate at N/100
(tests/golden/c4.json, made by oracle/gen_golden.py with the real reference binary) and finish
with exit status 0, run as batches of <= 50 separated by F lines -- the reference's protocol.
One step = the whole batch through libqe's product default: qe_run_queries_lanes with the
partitioned plan per query (the faithful executor for the queries it refuses) on concurrent lanes.

Multi-GPU: queries are independent, so the batch is scheduled replicas-style:
query i runs on rank i mod N, every rank holds every relation (1.8 GB), outputs are gathered to
rank 0 in input order.  Total work is fixed: strong scaling.
"""
from __future__ import annotations

import json
import os
import time

from qe import datagen as dg

from .cpuref import CpuRef, cpu_model, pin_one_core

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "c4.json")
GOLDEN_FULL = os.path.join(ROOT, "tests", "golden", "full", "c4_full.json")   # cpu_ref at full size
METRIC = "queries/sec, SIGMOD-2018-style batch (C4: 14 relations, gated query set)"


def load_queries() -> list[str]:
    with open(GOLDEN) as f:
        doc = json.load(f)
    return [c["input"] for c in doc["cases"] if c["rc"] == 0]


gen_c4 = dg.gen_c4


def cpu_sample(queries: list[str], gpu_ctx, budget_s: float = 20.0) -> dict:
    """oracle/cpu_ref, one core, on the first queries of the batch until ~budget_s of CPU time;
    the GPU runs the same queries one by one for a byte comparison."""
    specs = dg.c4_spec(1.0)
    cr = CpuRef()
    for cols in dg.make_relations(specs, dg.C4_SEED):
        cr.add_relation(cols)
    pin_one_core()
    done, cpu_outs, t_cpu = 0, [], 0.0
    for q in queries:
        out, _, dt = cr.run(q)
        t_cpu += dt
        cpu_outs.append(out)
        done += 1
        if t_cpu > budget_s:
            break
    cr.close()
    gpu_outs = [gpu_ctx.run(q)[0] for q in queries[:done]]
    return {"value": round(done / t_cpu, 3), "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"first {done} of {len(queries)} C4 queries at full size; oracle/cpu_ref single-threaded, "
                      f"{t_cpu:.1f} s",
            "seconds": round(t_cpu, 3), "queries": done, "cpu_model": cpu_model(), "parity_with_gpu": cpu_outs == gpu_outs}


def install_crash_maps():
    """QE_CRASH_MAPS=FILE: on SIGSEGV / SIGBUS append the fault address, PC and /proc/self/maps to
    FILE before the previous handler reports (tools/crashmaps.c; the profiled C4 runs' crash)."""
    if os.environ.get("QE_CRASH_MAPS"):
        import ctypes
        cm = ctypes.CDLL(os.path.join(ROOT, "query-compiler-executor_amd", "build", "libqecrash.so"))
        cm.qecrash_install.argtypes = [ctypes.c_char_p]
        if cm.qecrash_install(os.environ["QE_CRASH_MAPS"].encode()) != 0:
            raise RuntimeError("qecrash_install failed")


def run_single(args, log, roofline_fn=None, traffic_fn=None) -> dict:
    import torch

    from qe import lib
    torch.cuda.init()
    ctx = lib.Ctx(0)
    queries = load_queries()
    text = dg.c4_batches(queries)
    t0 = time.time()
    specs = gen_c4(ctx)
    log(f"[c4] {len(specs)} relations in HBM in {time.time() - t0:.2f}s; {len(queries)} gated queries")
    # the measured line: the batch's queries on concurrent lanes (qe_run_queries_lanes: worker
    # contexts on this GPU, each its own stream, the relations shared), each query through the
    # partitioned plan with the faithful executor for what it refuses; `--plan faithful` = the
    # faithful executor on the lanes
    workers = int(os.environ.get("QE_WORKERS", "8"))
    plan = getattr(args, "plan", "auto") != "faithful"
    install_crash_maps()
    # QE_BENCH_EVENTS=0: no HIP-event stage table on the lanes (the off switch ADVICE r4 asked to keep)
    events = os.environ.get("QE_BENCH_EVENTS", "1") != "0"

    def run_batch():
        return ctx.run_lanes(text, workers, plan=plan)

    def timed_batches():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = r = None
        for _ in range(args.steps):
            o, r = run_batch()
        ctx.sync()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, o, r

    out = None
    for _ in range(args.warmup):
        out, rc = run_batch()
    # 1) the stage table: every launch on every lane between two HIP events (round 3 switched them
    #    off under rocprofv3, where the lanes' event-query spins crashed inside the runtime; results
    #    now come back through a pinned flag -- qe_runtime.hip read_words -- with no runtime call in
    #    the wait).  Their host cost stretches a batch by ~16 % (r06u: 225 vs 189 ms), so this loop
    #    is not the one `value` comes from.
    stage_stats, dt_stages = {}, None
    if events:
        ctx.set_profiling(True)
        ctx.reset_stats()
        dt_stages, _, _ = timed_batches()
        stage_stats = ctx.kernel_stats()
        ctx.set_profiling(False)
    # 2) the timed region: HIP events around the dominant stage's launches only (its roofline), as
    #    on the C3 line
    dominant = max(((k, v) for k, v in stage_stats.items() if v["ms"] > 0), key=lambda kv: kv[1]["ms"],
                   default=(None, None))[0]
    if dominant:
        ctx.set_profiling_only(dominant)
        ctx.set_profiling(True)
    ctx.reset_stats()
    hits0, builds0 = ctx.sort_cache_stats()
    dt, out, rc = timed_batches()
    stats = ctx.kernel_stats() if dominant else {}
    ctx.set_profiling(False)
    ctx.set_profiling_only(None)
    hits1, builds1 = ctx.sort_cache_stats()
    kern = sorted(((k, v) for k, v in stage_stats.items() if not k.startswith("rt@")), key=lambda kv: -kv[1]["ms"])

    def timed(fn):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        o = fn()
        ctx.sync()
        d = time.perf_counter() - t1
        return {"ms_per_step": round(d * 1e3, 3), "value": round(len(queries) / d, 2), "stdout_identical": o == out}
    def no_cache(fn):   # the same lanes without the batch's shared base-column sorts
        os.environ["QE_SORT_CACHE"] = "0"
        try:
            return fn()
        finally:
            del os.environ["QE_SORT_CACHE"]
    others = {"plan_lanes_without_sort_cache (QE_SORT_CACHE=0)":
                  no_cache(lambda: timed(lambda: ctx.run_lanes(text, workers, plan=plan)[0])),
              "sequential_faithful (qe_run_queries)": timed(lambda: ctx.run(text)[0]),
              "partitioned_plan_one_lane (qe_run_queries_dist)": timed(lambda: ctx.run_dist(text)[0]),
              "faithful_lanes (qe_run_queries_parallel, %d lanes)" % workers:
                  timed(lambda: ctx.run_lanes(text, workers, plan=False)[0])}
    res = {
        "metric": METRIC, "value": round(len(queries) * args.steps / dt, 2), "unit": "queries/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: qe.datagen.c4_spec(1.0) relations generated in HBM (seed 4)",
        "parity": out == "".join(c["stdout"] for c in json.load(open(GOLDEN_FULL))["cases"])
                  if os.path.exists(GOLDEN_FULL) else None,
        "config": {"workload": "C4: 14 relations, %d gated SIGMOD-style queries in batches of %d"
                               % (len(queries), dg.C4_BATCH),
                   "rows_total": sum(s.rows for s in specs), "output_lines": out.count("\n"),
                   "executor": "qe_run_queries_lanes: %s, %d concurrent lanes (worker contexts = HIP "
                               "streams on this GPU, relations shared), output in input order"
                               % ("the partitioned plan per query, faithful fallback" if plan
                                  else "the faithful executor", workers),
                   "parallelism": "single GPU, inter-query concurrency x%d" % workers},
        "sort_cache": {"base_column_sorts_reused_per_step": (hits1 - hits0) / args.steps,
                       "built_per_step": (builds1 - builds0) / args.steps,
                       "scope": "one batch (qe_sort_cache brackets each qe_run_queries_lanes call): every step "
                                "sorts each base column it joins at least once"},
        "other_executors_same_batch": others,
        "roofline": roofline_fn(stats, traffic_fn() if traffic_fn else None) if roofline_fn else None,
        # (every lane's launches summed: lane time, ~3 kernels in flight at once)
        "stages_lane0": {k: {"ms_per_step": round(s["ms"] / args.steps, 3), "launches_per_step": s["launches"] / args.steps}
                   for k, s in kern[:10]},
        "stage_pass": None if dt_stages is None else {
            "ms_per_step": round(dt_stages / args.steps * 1e3, 3),
            "host_round_trips_per_step": stage_stats.get("host_round_trip", {}).get("launches", 0) / args.steps,
            "kernel_launches_per_step": sum(v["launches"] for k, v in stage_stats.items() if k != "host_round_trip") / args.steps,
            **({"round_trip_sites_per_step": {k[3:]: v["launches"] / args.steps for k, v in sorted(
                stage_stats.items(), key=lambda kv: -kv[1]["launches"]) if k.startswith("rt@")}}
               if any(k.startswith("rt@") for k in stage_stats) else {}),
            "note": "the stage table's own loop (HIP events around every launch on every lane); value's loop times "
                    "only the dominant stage"},
    }
    if not args.no_cpu:
        res["cpu_baseline"] = cpu_sample(queries, ctx)
    ctx.close()
    return res


def run_dist(args, log) -> dict | None:
    """replicas-style: rank r runs the r-th contiguous share of the batch on its own GPU (relations
    replicated), its queries on concurrent lanes (qe_run_queries_lanes, the plan per query with the
    faithful fallback); rank 0 joins the shares
    in rank order -- input order -- cut after the first share where the reference exits.
    torch.distributed (gloo) is the control plane only: barriers, the max time, the gather."""
    import torch
    import torch.distributed as dist

    from qe import lib
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    workers = int(os.environ.get("QE_WORKERS", "8"))
    ctx = lib.Ctx(dev)
    queries = load_queries()
    lo, hi = len(queries) * rank // world, len(queries) * (rank + 1) // world
    mine = "".join(queries[lo:hi])               # no F lines needed: one batch per rank
    gen_c4(ctx)
    res_mine = ("", 0)
    for _ in range(args.warmup):
        res_mine = ctx.run_lanes(mine, workers)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res_mine = ctx.run_lanes(mine, workers)
    ctx.sync()
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt = float(tmax.item())
    gathered = [None] * world
    dist.all_gather_object(gathered, res_mine)
    ctx.close()
    if rank != 0:
        return None
    text, rc = "", 0
    for out, r in gathered:
        text += out
        if r:
            rc = r
            break
    want = "".join(c["stdout"] for c in json.load(open(GOLDEN_FULL))["cases"]) if os.path.exists(GOLDEN_FULL) else None
    return {
        "metric": METRIC, "value": round(len(queries) * args.steps / dt, 2), "unit": "queries/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: qe.datagen.c4_spec(1.0) relations generated in HBM (seed 4), replicated on every rank",
        "parity": (text == want and rc == 0) if want is not None else None,
        "config": {"workload": "C4: 14 relations, %d gated SIGMOD-style queries" % len(queries),
                   "output_lines": text.count("\n"),
                   "executor": "qe_run_queries_lanes per rank (the plan per query, faithful fallback; %d "
                               "lanes), a contiguous share of the batch per rank" % workers,
                   "parallelism": f"query-parallel replicas x{world}"},
        "roofline": None, "cpu_baseline": None,
    }
