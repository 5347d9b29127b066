// VALU issue-rate probe for the roofline peak bench.py prices the traversal against: every SIMD runs
// `waves` waves of 64 lanes, each lane 8 independent v_fma_f32 chains (no dependent-latency stall);
// reports wave64 VALU instructions per SIMD per cycle at the measured clock (s_memtime / s_memrealtime).
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/valu_rate.hip -o tools/valu_rate (no v_pk_fma_f32)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define ITERS 4096
__global__ __launch_bounds__( 256 ) void k_fma( float* out, float a, float b, unsigned long long* clk )
{
	float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
	const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
	for (int i = 0; i < ITERS; i++)
	{
		x0 = __builtin_fmaf( x0, a, b ); x1 = __builtin_fmaf( x1, a, b ); x2 = __builtin_fmaf( x2, a, b ); x3 = __builtin_fmaf( x3, a, b );
		x4 = __builtin_fmaf( x4, a, b ); x5 = __builtin_fmaf( x5, a, b ); x6 = __builtin_fmaf( x6, a, b ); x7 = __builtin_fmaf( x7, a, b );
	}
	const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
	out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
	if (threadIdx.x == 0) clk[blockIdx.x * 2] = c1 - c0, clk[blockIdx.x * 2 + 1] = r1 - r0;
}

int main()
{
	hipDeviceProp_t p;
	hipGetDeviceProperties( &p, 0 );
	const int cus = p.multiProcessorCount;
	for (int wavesPerSimd : { 1, 2, 4, 8 })
	{
		const int blocks = cus * wavesPerSimd;   // 4 waves per block = one per SIMD
		float* out; unsigned long long* clk;
		hipMalloc( &out, (size_t)blocks * 256 * 4 );
		hipMalloc( &clk, (size_t)blocks * 16 );
		hipEvent_t e0, e1;
		hipEventCreate( &e0 ); hipEventCreate( &e1 );
		k_fma<<<blocks, 256>>>( out, 0.999f, 0.001f, clk );
		hipEventRecord( e0 );
		const int reps = 10;
		for (int r = 0; r < reps; r++) k_fma<<<blocks, 256>>>( out, 0.999f, 0.001f, clk );
		hipEventRecord( e1 );
		hipEventSynchronize( e1 );
		float ms; hipEventElapsedTime( &ms, e0, e1 );
		std::vector<unsigned long long> h( blocks * 2 );
		hipMemcpy( h.data(), clk, blocks * 16, hipMemcpyDeviceToHost );
		std::vector<double> ghz;
		for (int i = 0; i < blocks; i++) ghz.push_back( (double)h[2 * i] / ((double)h[2 * i + 1] / 100e6) / 1e9 );
		std::sort( ghz.begin(), ghz.end() );
		const double clock = ghz[ghz.size() / 2];
		const double insts = (double)blocks * 4 * ITERS * 8;          // wave64 v_fma_f32 per launch
		const double perSimd = insts / (cus * 4.0);
		const double cyc = ms / reps * 1e-3 * clock * 1e9;
		printf( "{\"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, \"wave_insts_per_simd_per_cycle\": %.4f, \"cycles_per_wave_inst\": %.3f}\n",
			wavesPerSimd, ms / reps, clock, perSimd / cyc, cyc / perSimd );
		hipFree( out ); hipFree( clk );
	}
	return 0;
}
