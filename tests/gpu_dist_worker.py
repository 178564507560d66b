"""Spawned rank for tests/test_gpu_dist.py: bench.py --workload c4 at N > 1, two ranks sharing the
box's one GPU under a gloo control plane.  TEST INFRASTRUCTURE."""
import os


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
