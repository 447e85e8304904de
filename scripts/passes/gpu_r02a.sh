#!/bin/bash
# Round-2 GPU check: gpu tests (new multi-rank + wide-split cases included),
# a 1-GPU bench line, and a 2-rank gloo rehearsal of the strong-scaling bench
# (both ranks on cuda:0).  Each GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu" && timeout -k 10 ${PYTEST_TIMEOUT:-700} python -u -m pytest tests -x -q -m "gpu${PYTEST_EXTRA:+ and $PYTEST_EXTRA}" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== bench" && timeout -k 10 300 python bench.py --cpu-budget 4 --config5 0 > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& echo "== bench 2-rank gloo rehearsal" && DN_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --config4-log2n 22 --allgather > gpurun_out/bench2_gloo.json 2> gpurun_out/bench2_gloo.err \
&& echo "== done"
rc=$?
tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
