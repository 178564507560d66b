# dist-plan checks on one GPU: primitive tests, the plans at N = 1 (no group), and 2-rank
# gloo rehearsals of the N > 1 code paths (both ranks on the one GPU, host-staged exchange)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_dist_tests.log 2>&1 && \
timeout -k 10 240 python bench.py --plan dist --steps 5 --warmup 2 --no-cpu > gpurun_out/dist_solo.log 2>&1 && \
QE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --rows 20000000 > gpurun_out/dist_gloo2.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c5 --plan dist --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_dist_solo.log 2>&1
echo rc=$?
