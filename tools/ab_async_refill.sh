set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/async
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/async/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/async/tests.log; exit 1; }
tail -1 gpurun_out/async/tests.log
for rep in 1 2; do
 for cfg in "sync 48" "new 48" "new 40" "new 32" "new 24" "new 16"; do
  set -- $cfg
  if [ $1 = sync ]; then export LH2_CORE_LIB=$GRAFT_REPO_ROOT/gpuab/sync/libRenderCore_MI355X.so; else unset LH2_CORE_LIB; fi
  timeout -k 10 150 python3 tools/trace_kernel_bench.py --set both --iters 20 --refill $2 > gpurun_out/async/c.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/async/c.log') if l.startswith('{')][-1])
print('$1 refill $2', 'primary', d['primary']['ms'], 'bounce', d['bounce']['ms'])"
 done
done
