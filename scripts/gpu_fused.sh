#!/bin/bash
# Fused-Adam / split-K fixup check: focused GPU tests, then the full GPU suite, then a bench A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-fused}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_adam_gpu.py > $O/t_fused.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $O/t_fused.log | head -30; [ $rc -ne 0 ] && { tail -30 $O/t_fused.log; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
bash scripts/gpu_ab.sh ${1:-fused}/ab "" "--no-fused-adam" ${2:-2}
