"""Spawned rank for tests/test_gpu_dist.py: the C5 aggregate plan on the real GPUEngine (libqe)
under gloo, two ranks sharing the box's one GPU (host-staged all-reduce).  TEST INFRASTRUCTURE."""
import os


def agg_worker(rank, world, port, rows, queries, outq):
    """the aggregate (skew) plan on C5-shaped data, `rows` per side"""
    import torch
    import torch.distributed as dist

    from qe import datagen as dg
    from qe import lib
    from qe.dist import DistAggJoin, GPUEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ctx = lib.Ctx(0)
    try:
        dg.gen_c5(ctx, rows)
        ex = DistAggJoin(GPUEngine(ctx, rank, world), [rows, rows])
        res = [ex.run(q) for q in queries]
        if rank == 0:
            outq.put(res)
    finally:
        ctx.close()
        dist.destroy_process_group()


def c4_worker(rank, world, port, outq):
    """one rank of bench.py --workload c4 at N > 1 (benchmarks/c4.run_dist), all ranks on the one GPU"""
    import sys
    import types
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", QE_WORKERS="3")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from benchmarks import c4
    res = c4.run_dist(types.SimpleNamespace(steps=1, warmup=0), print)
    if rank == 0:
        outq.put(res)
