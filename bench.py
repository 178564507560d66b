#!/usr/bin/env python3
"""bench.py -- the headline benchmark: joined tuples/s on the 4-relation chain join (config C3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--no-cpu] [--workload c3|c4|c5]

Workload (BASELINE.json configs[2]): four relations of R = 100 M rows
(c0 = v % R, c1 = v % R, c2 = v >> 32, splitmix64 seed 1, generated straight into HBM), query
    0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2
One step = one full execution of that query: both filters, three sort-merge joins, the
mid_result payload propagation and the three checksums, printed exactly as the reference
prints them.  `value` = chain rows produced per second (joined tuples/s), whole job.

Every N runs libqe's partitioned executor, qe_run_queries_dist (host C, include/qe_plan.h): a
replay of the reference's mid_result state machine on the bindings decides that this query's
output is the relational answer, so it runs as a relational plan --
filters on rowid slices, joins reordered smallest-first, each join a sort-merge on its key buckets
(qe_join_pairs), derived join sides exchanged by key over RCCL at N > 1 (grouped
ncclSend/ncclRecv on the communicator's stream), sums all-reduced -- and prints the reference's
bytes.  At N = 1 the faithful executor (qe_run_queries: the reference's state machine restated,
every mid_result list kept) is timed in the same run and reported as `faithful_executor`
(`--plan faithful` makes it the measured line).
`--scaling strong` (default, the north star's shape): 100 M rows per relation in total, whatever N;
`--scaling weak`: 100 M rows per relation per GPU.  Rank 0 checks the printed bytes in-run against
the faithful executor on the same relations (and, for the default workload, against the C3 output
pinned by tests/test_gpu_fullsize.py::test_c3_chain_100m) and reports `parity`.

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
# C3 at 100 M rows/relation, seed 1: the bytes tests/test_gpu_fullsize.py::test_c3_chain_100m pins
# against the aggregate truth (itself pinned to the reference's G1-G3 goldens)
C3_100M_STDOUT = "46567055\n100034367840717139 100020175372851973 93168255049607962 \n"
QUERY = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_chain(ctx, rows: int, seed: int, key_domain: int, row_start: int = 0):
    kinds = [("mod", key_domain), ("mod", key_domain), ("hi32",)]
    return [ctx.gen_relation(rows, kinds, seed=seed, gen_rel=r, row_start=row_start) for r in range(4)]


def roofline(stats: dict, traffic: dict | None, steps: int | None = None):
    """the dominant stage: algorithmic bytes per launch / mean launch time (HIP events), and its
    PMC traffic per launch = the stage's PMC bytes per query / its launches per step (`steps` =
    queries behind `stats`) -- both sides over the same launch set"""
    if not stats:
        return None
    name, s = max(stats.items(), key=lambda kv: kv[1]["ms"])
    per_launch_ms = s["ms"] / max(1, s["launches"])
    per_launch_bytes = s["alg_bytes"] / max(1, s["launches"])
    achieved = per_launch_bytes / (per_launch_ms * 1e-3) / 1e9 if per_launch_ms > 0 else 0.0
    t = None
    if traffic and name in traffic:
        tq = traffic[name].get("per_query")
        if tq and steps and s["launches"]:
            t = round(tq / (s["launches"] / steps))
        elif tq is None:
            t = traffic[name].get("per_dispatch")      # workloads profiled without a query count
    return {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": t,
            "alg_bytes_per_launch": per_launch_bytes, "avg_launch_ms": round(per_launch_ms, 4),
            "launches": s["launches"]}


def stage_roofline(stats: dict, traffic: dict | None, steps: int) -> dict:
    """every stage against the same roofline; `traffic_over_alg` = the stage's PMC bytes per query
    (all of its dispatches) / its algorithmic bytes per step (all of its `Timed` launches) -- a
    per-query ratio, so a stage whose timer spans several dispatches is not misreported"""
    out = {}
    for name, s in sorted(stats.items(), key=lambda kv: -kv[1]["ms"]):
        if not s["launches"] or s["ms"] <= 0 or not s["alg_bytes"]:
            continue
        per_ms = s["ms"] / s["launches"]
        per_b = s["alg_bytes"] / s["launches"]
        gbs = per_b / (per_ms * 1e-3) / 1e9
        tq = (traffic.get(name) or {}).get("per_query") if traffic else None
        alg_q = s["alg_bytes"] / steps
        out[name] = {"launches": s["launches"], "avg_launch_ms": round(per_ms, 4), "alg_gb_per_launch": round(per_b / 1e9, 4),
                     "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 3),
                     "alg_gb_per_query": round(alg_q / 1e9, 4),
                     "pmc_gb_per_query": round(tq / 1e9, 4) if tq else None,
                     "traffic_over_alg": round(tq / alg_q, 3) if tq else None}
    return out


def infer_queries(command: str):
    """queries a profiled `bench.py` c3 plan command ran: warmup + 2 x steps (the stage-table loop
    and the timed loop; tools/pmc_traffic.py records it as "queries" from round 4 on)"""
    import re
    m_s = re.search(r"--steps (\d+)", command or "")
    m_w = re.search(r"--warmup (\d+)", command or "")
    if not m_s or "bench.py" not in command or "--workload c4" in command or "--workload c5" in command:
        return None
    return (int(m_w.group(1)) if m_w else 2) + 2 * int(m_s.group(1))


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
        q = d.get("queries") or infer_queries(d.get("command", ""))
        out = {}
        for k, v in d.get("kernels", {}).items():
            pq = v.get("hbm_bytes_per_query")
            if pq is None and q and v.get("launches_fetch_pass"):
                pq = v["hbm_bytes_per_launch"] * v["launches_fetch_pass"] / q
            out[k] = {"per_dispatch": v.get("hbm_bytes_per_launch"), "per_query": pq}
        out["_file"] = os.path.relpath(path, ROOT)
        return out
    return None


def cpu_baseline(sample_rows: int, seed: int, gpu_ctx):
    """oracle/cpu_ref (single thread) on a bounded sample of the same workload; the GPU runs
    the same sample so the two outputs are compared bit for bit."""
    from benchmarks.cpuref import CpuRef, cpu_model, pin_one_core
    from qe import datagen as dg
    cr = CpuRef()
    for cols in dg.make_relations(dg.chain_spec(4, sample_rows), seed):
        cr.add_relation(cols)
    pin_one_core()
    cpu_out, rc, dt = cr.run(QUERY)
    cr.close()
    # same sample on the GPU, for a bit-exact comparison
    gpu_ctx.drop_relations()
    gen_chain(gpu_ctx, sample_rows, seed, sample_rows)
    gpu_out, _ = gpu_ctx.run(QUERY)
    rows = gpu_ctx.last_result_rows()
    gpu_ctx.drop_relations()
    return {"value": round(rows / dt, 1), "unit": "joined tuples/s", "cores": 1, "kind": "port",
            "sample": f"C3 shape at {sample_rows} rows/rel (seed {seed}); oracle/cpu_ref single-threaded, "
                      f"{dt:.2f} s for {rows} chain rows",
            "seconds": round(dt, 3), "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "parity_with_gpu": cpu_out == gpu_out and rc == 0, "sample_stdout": cpu_out}


def pinned_parity(args, out):
    """the printed bytes against the pinned C3 output (default workload only; None otherwise)"""
    if args.rows == 100_000_000 and args.seed == 1:
        return out == C3_100M_STDOUT
    return None


def run_dist(args):
    """the partitioned plan (C, include/qe_plan.h) on every rank of an RCCL communicator"""
    import torch
    import torch.distributed as dist

    from qe import lib
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    torch.cuda.init()
    multi = world > 1
    if multi and not dist.is_initialized():
        dist.init_process_group("gloo")          # control plane only: the bootstrap id, barriers, max time
    ctx = lib.Ctx(dev)
    comm = None
    if multi:
        box = [lib.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        comm = lib.Comm(ctx, world, rank, box[0])   # the data path: RCCL over xGMI
    total = args.rows if args.scaling == "strong" else args.rows * world
    t0 = time.time()
    gen_chain(ctx, total, args.seed, total)       # replicated on every rank
    ctx.sync()
    t_part = None
    if multi:   # partitioned layout: a join-key column's hash bucket is kept from its first use (warmup)
        t1 = time.time()
        ctx.partition_columns(world, rank)
        t_part = time.time() - t1
    if rank == 0:
        log(f"[bench] {world} rank(s): 4 x {total} rows x 3 cols in HBM per GPU in {time.time() - t0:.2f}s"
            + (f" (partitioned in {t_part:.3f}s)" if t_part is not None else ""))
    out = None
    for i in range(args.warmup):
        out, _, refused = ctx.run_dist(QUERY, comm)
        if rank == 0:
            log(f"[bench] warmup {i}: {out.strip()!r} (refused {refused})")

    def timed_steps():
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = rc_ = rf = None
        for _ in range(args.steps):
            o, rc_, rf = ctx.run_dist(QUERY, comm)
        ctx.sync()
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        d = time.perf_counter() - t0
        if multi:
            t = torch.tensor([d], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d = float(t.item())
        return d, o, rc_, rf

    # 1) the stage table: every launch between two HIP events (their host cost stretches the
    #    wall time, so this loop is not the one `value` comes from)
    ctx.set_profiling(True)
    ctx.reset_stats()
    dt_stages, _, _, _ = timed_steps()
    stage_stats = ctx.kernel_stats()
    ctx.set_profiling(False)
    # QE_RT_SITES=1: the host round trips by call site (zero-time stages "rt@file:line")
    rt_sites = {k[3:]: stage_stats.pop(k)["launches"] / args.steps for k in
                [k for k in stage_stats if k.startswith("rt@")]}
    dominant = max(((k, v) for k, v in stage_stats.items() if v["ms"] > 0), key=lambda kv: kv[1]["ms"])[0]
    # 2) the timed region: HIP events around the dominant kernel's launches only (its roofline)
    ctx.set_profiling_only(dominant)
    ctx.set_profiling(True)
    ctx.reset_stats()
    dt, out, rc, refused = timed_steps()
    stats = ctx.kernel_stats()
    ctx.set_profiling(False)
    ctx.set_profiling_only(None)
    rows = ctx.last_result_rows()
    exchanges, sent = comm.stats() if comm else (0, 0)
    res = None
    faithful_line = None
    faithful = None
    if rank == 0 and not args.no_faithful:
        faithful, _ = ctx.run(QUERY)              # in-run parity: the drop-in executor, same relations
    # 3) the same plan with the query's last join materialised (QE_PLAN_AGG=0: its pairs made by the
    #    chain bucket join, then summed by the checksum gathers) -- the line's own last join counts
    #    its pairs in aggregate form and never writes them; every rank runs it (it is collective)
    def timed_with(var, val):
        """the timed loop with one switch flipped, after its own untimed warmup (a form's first
        queries allocate the buffers its allocator then reuses)"""
        old = os.environ.get(var)
        os.environ[var] = val
        try:
            for _ in range(max(1, args.warmup)):
                ctx.run_dist(QUERY, comm)
            return timed_steps()
        finally:
            if old is None:
                del os.environ[var]
            else:
                os.environ[var] = old

    mat_line = side_line = None
    if not args.no_materialised and not args.no_faithful:   # (profiling runs: the measured plan only)
        dtm, out_m, _, _ = timed_with("QE_PLAN_AGG", "0")
        mat_line = {"last_join": "materialised: every result pair written (rowid pairs + carried columns), "
                                 "then the checksums gather the select columns",
                    "ms_per_step": round(dtm / args.steps * 1e3, 3),
                    "value": round(ctx.last_result_rows() * args.steps / dtm, 1),
                    "stdout_identical": out_m == out}
        # 4) the same plan with each join's two sorts on two streams (QE_SIDE_STREAM=1, SideFork):
        #    faster end to end, but its kernels share the GPU, so the line's per-launch roofline is
        #    measured with it off (the default)
        if os.environ.get("QE_SIDE_STREAM", "0") != "1":
            dts, out_s, _, _ = timed_with("QE_SIDE_STREAM", "1")
            side_line = {"side_stream": "one join side's sort on a second HIP stream beside the other's",
                         "ms_per_step": round(dts / args.steps * 1e3, 3),
                         "value": round(ctx.last_result_rows() * args.steps / dts, 1),
                         "stdout_identical": out_s == out}
    if rank == 0:
        if faithful is not None and not multi:   # N = 1: the faithful executor timed too, for the record
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                ctx.run(QUERY)
            ctx.sync()
            torch.cuda.synchronize()
            dtf = time.perf_counter() - t1
            faithful_line = {"executor": "qe_run_queries (the reference's state machine restated, every "
                                         "mid_result list kept as it keeps them)",
                             "ms_per_step": round(dtf / args.steps * 1e3, 3),
                             "value": round(ctx.last_result_rows() * args.steps / dtf, 1),
                             "stdout_identical": faithful == out}
        kern = sorted(stage_stats.items(), key=lambda kv: -kv[1]["ms"])
        traffic = load_traffic("c3_plan")
        res = {
            "metric": METRIC, "value": round(rows * args.steps / dt, 1), "unit": "joined tuples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "dtype": "u64",
            "data": "synthetic: splitmix64 relations generated in HBM on every rank (SURVEY.md §9.1), seed %d"
                    % args.seed,
            "parity": (faithful is None or out == faithful) and pinned_parity(args, out) is not False,
            "parity_detail": {"equals_faithful_executor": None if faithful is None else out == faithful,
                              "equals_pinned_c3_100m": pinned_parity(args, out)},
            "config": {"workload": "C3: 4-relation chain join, 2 filters on R3, %d rows/rel in total" % total,
                       "query": QUERY.strip(), "rows_per_relation": total, "result_rows": rows, "stdout": out,
                       "executor": "qe_run_queries_dist: host-C partitioned plan (include/qe_plan.h), "
                                   "RCCL grouped send/recv per exchange, all-reduced sums",
                       "refused_queries": refused, "exchanges_per_step": exchanges / max(1, args.steps + args.warmup),
                       "parallelism": f"hash-partitioned dp{world}" if multi else "partitioned plan, one rank",
                       "last_join": "aggregate (the last join's pairs counted, not materialised: only "
                                    "print_sums reads them; see materialised_last_join)",
                       "load_partition_s": round(t_part, 4) if t_part is not None else None},
            "materialised_last_join": mat_line,
            "two_stream_sorts": side_line,
            "faithful_executor": faithful_line,
            "roofline": roofline({dominant: stats[dominant]} if dominant in stats else stats,
                                 traffic, args.steps),
            # the stage table's loop (every launch timed): kernel time and host round trips per step
            "kernel_ms_per_step": round(sum(s["ms"] for _, s in kern) / args.steps, 3),
            "host_round_trips_per_step": stage_stats.get("host_round_trip", {}).get("launches", 0) / args.steps,
            **({"round_trip_sites_per_step": dict(sorted(rt_sites.items(), key=lambda kv: -kv[1]))} if rt_sites else {}),
            "stage_table_loop_ms_per_step": round(dt_stages / args.steps * 1e3, 3),
            "stages": {k: {"ms_per_step": round(s["ms"] / args.steps, 3)} for k, s in kern[:12]},
            # every stage against the same roofline (algorithmic bytes per launch / mean launch time
            # of the stage-table loop), with its PMC traffic ratio where profiles/ has one
            "stage_roofline": stage_roofline(stage_stats, traffic, args.steps),
            "pmc_source": traffic.get("_file") if traffic else None,
        }
        if not args.no_cpu and not multi:   # (rank 0 at N = 1 only: the baseline is per host, not per rank)
            res["cpu_baseline"] = cpu_baseline(args.cpu_rows, args.seed, ctx)
        else:
            res["cpu_baseline"] = None
    if multi:
        dist.barrier()
    if comm:
        comm.close()
    ctx.close()
    if multi:
        dist.destroy_process_group()
    return res


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
        "scaling": args.scaling, "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: splitmix64 relations generated in HBM (SURVEY.md §9.1), seed %d" % args.seed,
        "parity": pinned_parity(args, out),
        "config": {"workload": "C3: 4-relation chain join R0-R1-R2-R3, 2 filters on R3, %d rows/rel" % args.rows,
                   "query": QUERY.strip(), "rows_per_relation": args.rows, "result_rows": rows,
                   "stdout": out, "executor": "libqe faithful state machine (qe_run_queries)",
                   "dead_list_elimination": os.environ.get("QE_DLE", "1") != "0",
                   "parallelism": "single GPU"},
        "all_lists_materialised": {"ms_per_step": round(dt_all / args.steps * 1e3, 3),
                                   "value": round(rows * args.steps / dt_all, 1),
                                   "stdout_identical": out_all == out},
        "roofline": roofline(stats, load_traffic(), args.steps),
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


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` with no launcher around us: start N rank processes of this script (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set, one per GPU) and relay rank 0's JSON line.  This
    process never imports torch nor touches a GPU (a GPU-initialised process must not spawn the
    ranks' runtimes under it); a rank that exits non-zero ends the others and the launch."""
    import subprocess
    import tempfile
    port = free_port()
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), QE_BENCH_LAUNCHER="bench.py")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                      stdout=out0 if r == 0 else sys.stderr))
    rc = 0
    try:
        while True:
            live = [p for p in procs if p.poll() is None]
            bad = [p for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                log(f"[bench] rank {procs.index(bad[0])} exited with status {rc}; stopping the other ranks")
                break
            if not live:
                break
            time.sleep(0.2)
    finally:
        for p in procs:                       # only the processes started here, by their Popen handles
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc:
        return rc if rc > 0 else 1
    out0.seek(0)
    lines = [ln for ln in out0.read().splitlines() if ln.strip()]
    ours = [ln for ln in lines if ln.startswith("{")]
    for ln in lines:                          # gloo's own chatter on rank 0's stdout goes to stderr
        if not ln.startswith("{"):
            log(ln)
    for ln in ours:
        print(ln, flush=True)
    return 0 if ours else 1


def check_world(args) -> tuple[int, int, int]:
    """(rank, world, local_rank) of this process; exits non-zero when the launch does not match
    `--gpus` or when this node has fewer GPUs than ranks (never a silent one-rank line)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
        sys.exit(2)
    if not args.dry_launch:
        import torch
        ngpu = torch.cuda.device_count()           # counting devices does not initialise them
        if ngpu < world:
            log(f"[bench] error: --gpus {world} but this node shows {ngpu} GPU(s); one rank per GPU is required")
            sys.exit(3)
    return rank, world, local


def dry_launch(args):
    """--dry-launch: every rank joins the gloo control plane and stops before any GPU work; rank 0
    prints what the launch produced (the CPU test of the launcher)."""
    import torch.distributed as dist
    rank, world, local = check_world(args)
    if world > 1:
        dist.init_process_group("gloo")
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "local_rank": local, "pid": os.getpid()})
        dist.barrier()
        dist.destroy_process_group()
    else:
        got = [{"rank": 0, "local_rank": 0, "pid": os.getpid()}]
    if rank == 0:
        return {"dry_launch": True, "world_size": world, "gpus": args.gpus, "workload": args.workload,
                "launcher": os.environ.get("QE_BENCH_LAUNCHER", "external" if "WORLD_SIZE" in os.environ else "none"),
                "ranks": got}
    return None


SCALE_NOTE = ("N > 1 runs one rank process per GPU (bench.py starts them itself, or runs under "
              "torch.distributed.run); no 1/2/4/8-GPU curve has been measured by this build's author "
              "(1-GPU pool) -- the N > 1 path was exercised with in-process ranks on one GPU")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks = GPUs of this node (default: $WORLD_SIZE or 1); without a launcher, N > 1 "
                         "starts N rank processes of this script")
    ap.add_argument("--dry-launch", action="store_true",
                    help="start the ranks, join the gloo control plane, stop before any GPU work (launcher test)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=None,
                    help="rows per relation (per rank for N > 1); default 1e8 (c3) / 1e9 (c5)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-rows", type=int, default=16_000_000)
    ap.add_argument("--cpu-rows-c5", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-faithful", action="store_true",
                    help="skip the faithful executor's parity run and timing and the materialised-last-join "
                         "timing (profiling runs: only the measured executor's kernels in the trace)")
    ap.add_argument("--no-materialised", action="store_true",
                    help="c3: skip the materialised-last-join timing (QE_PLAN_AGG=0) reported beside the line")
    ap.add_argument("--workload", choices=["c3", "c4", "c5"], default="c3",
                    help="c3 (default): the headline 4-relation chain join; c4: the SIGMOD-style batch; "
                         "c5: the skewed (Zipf 0.9) 2-relation join at 1e9 rows")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="c3 at N > 1: strong = --rows per relation in total (the north star: 100 M), "
                         "weak = --rows per relation per GPU")
    ap.add_argument("--plan", choices=["auto", "dist", "faithful"], default="auto",
                    help="c3: auto / dist = qe_run_queries_dist, the partitioned executor, at every N (its "
                         "faithful fallback for queries outside the relational domain; at N = 1 the faithful "
                         "executor is timed beside it); faithful = qe_run_queries alone (N = 1); c5: dist = "
                         "the aggregate plan at N = 1 too")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world or "1")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.dry_launch:
        res = dry_launch(args)
        if res is not None:
            print(json.dumps(res), flush=True)
        return
    _, world, _ = check_world(args)
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
    elif args.plan == "faithful" and world == 1:
        res = run_single(args)
    else:
        res = run_dist(args)
    if res is not None:
        res["launcher"] = os.environ.get("QE_BENCH_LAUNCHER", "external (WORLD_SIZE set)" if env_world else "none")
        res["scale_note"] = SCALE_NOTE
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
