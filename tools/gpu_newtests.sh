# round-2 parity additions on one MI355X: the join_payloads limit, every golden through the drop-in
# binary, C4 at full size against cpu_ref's fixture, C5 at 1e9 rows against sharded torch truth
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_primitives.py::test_join_payloads_beyond_the_materialisation_limit_is_etoobig \
  tests/test_gpu_fullsize_batch.py > gpurun_out/newtests.log 2>&1
echo rc=$?
