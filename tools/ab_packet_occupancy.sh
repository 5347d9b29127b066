set -uo pipefail
export LH2_BLUENOISE=$PWD/lighthouse2_amd/data/bluenoise.bin
mkdir -p gpurun_out
for rep in 1 2; do for v in ${VARIANTS:-base p6 p7}; do
  LH2_CORE_LIB=$PWD/gpuvar/$v/libRenderCore_MI355X.so timeout -k 10 120 python3 tools/trace_kernel_bench.py --set primary --setting unitCoherent=1 > gpurun_out/abp_${v}_$rep.json 2>/dev/null || exit 1
done; done
