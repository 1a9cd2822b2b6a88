#!/bin/bash
# Targeted GPU tests, then N headline benches (no quality protocol) and a kernel-stats profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-check}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_dw_batch_gpu.py tests/test_fused_adam_gpu.py tests/test_prune_gpu.py tests/test_packed_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -B3 -A25 "Error\|assert" $O/tests.log | head -50; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-quality > $O/bench_$i.log 2>&1 || { tail -5 $O/bench_$i.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$i.log').read().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'], d['mean_loss'])"
done
bash scripts/gpu_prof_quick.sh $(basename $O)_prof
