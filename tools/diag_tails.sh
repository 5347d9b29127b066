set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
mkdir -p gpurun_out/diag
bash tools/valu_rate_pmc.sh > gpurun_out/diag/valu.log 2>&1 || exit 1
bash tools/share_timeline.sh 8 > gpurun_out/diag/share8.txt 2>&1 || exit 1
LH2_CORE_LIB=$ROOT/gpuab/tt/libRenderCore_MI355X.so LH2_TRACE_TIMES_OUT=$ROOT/gpurun_out/diag/tt_bounce.bin timeout -k 10 200 python3 tools/trace_kernel_bench.py --set bounce --iters 1 > gpurun_out/diag/tt.json 2>&1 || exit 1
python3 tools/trace_times.py gpurun_out/diag/tt_bounce.bin > gpurun_out/diag/tt.txt 2>&1
LH2_CORE_LIB=$ROOT/gpuab/ts/libRenderCore_MI355X.so timeout -k 10 200 python3 tools/trace_kernel_bench.py --set bounce --iters 1 > gpurun_out/diag/ts.json 2> gpurun_out/diag/ts.err || exit 1
echo diag done
