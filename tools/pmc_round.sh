#!/bin/bash
# Counter passes behind bench.py's roofline (run through gpurun from the repo root, after profile_gpu.sh):
#   sq1, sq2  SQ instruction-issue counters of the dominant kernel (k_trace_closest<false, 4> on the
#             config-2 bounce rays, tools/trace_kernel_bench.py --set bounce) + GRBM_GUI_ACTIVE (clock)
#   pk1       the same for the primary-ray launch (packet traversal, k_trace_closest_packet)
#   c5_fetch, c5_write  FETCH_SIZE / WRITE_SIZE over config-5 frames (10M triangles: the DRAM-real
#             working set), one TCC counter group per pass
#   c5_sq1, c5_sq2   the SQ sets over config-5 frames (its per-ray closest-hit launches)
#   c3_sq1, c3_sq2, c3_fetch, c3_write   the same over config-3 frames (the lit path: any-hit shadow launch,
#             lit shade, path tail)
# One --pmc pass per rocprofv3 run; each run under its own kill-timeout; chained with &&.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -f csv -d "$OUT/sq1" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 5 > "$OUT/sq1.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS \
    -f csv -d "$OUT/sq2" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 5 > "$OUT/sq2.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -f csv -d "$OUT/pk1" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set primary --iters 5 > "$OUT/pk1.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE \
    -f csv -d "$OUT/c5_fetch" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 5 --frames 3 --warmup 1 > "$OUT/c5_fetch.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE \
    -f csv -d "$OUT/c5_write" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 5 --frames 3 --warmup 1 > "$OUT/c5_write.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -f csv -d "$OUT/c5_sq1" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 5 --frames 3 --warmup 1 > "$OUT/c5_sq1.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS \
    -f csv -d "$OUT/c5_sq2" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 5 --frames 3 --warmup 1 > "$OUT/c5_sq2.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -f csv -d "$OUT/c3_sq1" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 3 --frames 5 --warmup 1 > "$OUT/c3_sq1.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS \
    -f csv -d "$OUT/c3_sq2" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 3 --frames 5 --warmup 1 > "$OUT/c3_sq2.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE \
    -f csv -d "$OUT/c3_fetch" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 3 --frames 5 --warmup 1 > "$OUT/c3_fetch.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE \
    -f csv -d "$OUT/c3_write" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 3 --frames 5 --warmup 1 > "$OUT/c3_write.log" 2>&1
echo "pmc round done"
