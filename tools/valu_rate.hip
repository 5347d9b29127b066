// VALU issue-rate probe for the roofline peak bench.py prices the traversal against: every SIMD runs
// `waves` waves of 64 lanes, each lane 8 independent chains (no dependent-latency stall); reports wave64
// VALU instructions per SIMD per cycle at the measured clock (s_memtime / s_memrealtime).
// Three instruction mixes (--mode, default all):
//   fma    v_fma_f32 only (8 per iteration, exact count);
//   pkfma  v_pk_fma_f32 only (8 per iteration, exact count: two FP32 FMAs per lane each);
//   mix    the BVH4 node step's mix: packed FMA slab planes, max3 / min3, compares, selects, integer key
//          and / or, unsigned min / max. Its count per iteration is the compiler's: run the probe under
//          `rocprofv3 --pmc SQ_INSTS_VALU` (tools/valu_rate_pmc.sh) and divide; the line carries
//          "insts_per_iter": null for that mode.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>

#define ITERS 4096
typedef float f2 __attribute__( (ext_vector_type( 2 )) );

__device__ inline void clocks( unsigned long long& c, unsigned long long& r ) { c = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__( 256 ) void k_fma( float* out, float a, float b, unsigned long long* clk )
{
	float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
	unsigned long long c0, r0, c1, r1;
	clocks( c0, r0 );
	for (int i = 0; i < ITERS; i++)
	{
		x0 = __builtin_fmaf( x0, a, b ); x1 = __builtin_fmaf( x1, a, b ); x2 = __builtin_fmaf( x2, a, b ); x3 = __builtin_fmaf( x3, a, b );
		x4 = __builtin_fmaf( x4, a, b ); x5 = __builtin_fmaf( x5, a, b ); x6 = __builtin_fmaf( x6, a, b ); x7 = __builtin_fmaf( x7, a, b );
	}
	clocks( c1, r1 );
	out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
	if (threadIdx.x == 0) clk[blockIdx.x * 2] = c1 - c0, clk[blockIdx.x * 2 + 1] = r1 - r0;
}

/* v_pk_fma_f32 on VGPR pairs; the asm pins the instruction form (the compiler would otherwise be free to
   split it into two v_fma_f32) */
#define PKFMA( x ) asm volatile( "v_pk_fma_f32 %0, %0, %1, %2" : "+v"( x ) : "v"( a2 ), "v"( b2 ) )
__global__ __launch_bounds__( 256 ) void k_pkfma( float* out, float a, float b, unsigned long long* clk )
{
	const f2 a2 = { a, a }, b2 = { b, b };
	f2 x0 = { (float)threadIdx.x, 1.0f }, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
	unsigned long long c0, r0, c1, r1;
	clocks( c0, r0 );
	for (int i = 0; i < ITERS; i++)
	{
		PKFMA( x0 ); PKFMA( x1 ); PKFMA( x2 ); PKFMA( x3 ); PKFMA( x4 ); PKFMA( x5 ); PKFMA( x6 ); PKFMA( x7 );
	}
	clocks( c1, r1 );
	const f2 s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
	out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
	if (threadIdx.x == 0) clk[blockIdx.x * 2] = c1 - c0, clk[blockIdx.x * 2 + 1] = r1 - r0;
}
#undef PKFMA

/* the node step's instruction mix per chain and iteration: two packed slab-plane FMAs, an entry max3 and an
   exit min3, the padded exit (fma), two compares and a select into an integer sort key (and / or), and an
   unsigned min / max compare-exchange against the chain's running keys; 8 independent chains */
__global__ __launch_bounds__( 256 ) void k_mix( float* out, float a, float b, unsigned long long* clk )
{
	const f2 a2 = { a, a }, b2 = { b, -b };
	f2 p[8];
	float m[8];
	uint32_t lo[8], hi[8];
	for (int c = 0; c < 8; c++) p[c] = (f2){ (float)threadIdx.x + c, (float)c }, m[c] = 0.5f * c, lo[c] = 0xffffffffu, hi[c] = 0;
	unsigned long long c0, r0, c1, r1;
	clocks( c0, r0 );
	for (int i = 0; i < ITERS; i++)
	{
#pragma unroll
		for (int c = 0; c < 8; c++)
		{
			f2 q;
			asm volatile( "v_pk_fma_f32 %0, %1, %2, %3" : "=v"( q ) : "v"( p[c] ), "v"( a2 ), "v"( b2 ) );
			asm volatile( "v_pk_fma_f32 %0, %0, %1, %2" : "+v"( p[c] ) : "v"( a2 ), "v"( b2 ) );
			const float tn = __builtin_fmaxf( __builtin_fmaxf( q.x, p[c].x ), m[c] );
			const float tf = __builtin_fmaf( __builtin_fminf( __builtin_fminf( q.y, p[c].y ), b ), 1.00001f, 1e-30f );
			const bool h = tn <= tf && tn <= a;
			const uint32_t k = h ? ((__float_as_uint( tn ) & 0x7ffff3ffu) | 0x400u) : 0xffffffffu;
			const uint32_t l = lo[c] < k ? lo[c] : k, u = lo[c] < k ? k : lo[c];
			lo[c] = l, hi[c] ^= u;
			m[c] = tf;
		}
	}
	clocks( c1, r1 );
	float s = 0;
	for (int c = 0; c < 8; c++) s += p[c].x + p[c].y + m[c] + (float)(lo[c] ^ hi[c]);
	out[blockIdx.x * blockDim.x + threadIdx.x] = s;
	if (threadIdx.x == 0) clk[blockIdx.x * 2] = c1 - c0, clk[blockIdx.x * 2 + 1] = r1 - r0;
}

typedef void (*KernelFn)( float*, float, float, unsigned long long* );

int main( int argc, char** argv )
{
	const char* only = argc > 2 && !strcmp( argv[1], "--mode" ) ? argv[2] : nullptr;
	hipDeviceProp_t p;
	hipGetDeviceProperties( &p, 0 );
	const int cus = p.multiProcessorCount;
	struct { const char* name; KernelFn fn; int insts; } modes[] = { { "fma", k_fma, 8 }, { "pkfma", k_pkfma, 8 }, { "mix", k_mix, 0 } };
	for (auto& md : modes)
	{
		if (only && strcmp( only, md.name )) continue;
		for (int wavesPerSimd : { 1, 2, 4, 8 })
		{
			const int blocks = cus * wavesPerSimd;   // 4 waves per block = one per SIMD
			float* out; unsigned long long* clk;
			hipMalloc( &out, (size_t)blocks * 256 * 4 );
			hipMalloc( &clk, (size_t)blocks * 16 );
			hipEvent_t e0, e1;
			hipEventCreate( &e0 ); hipEventCreate( &e1 );
			md.fn<<<blocks, 256>>>( out, 0.999f, 0.001f, clk );
			hipEventRecord( e0 );
			const int reps = 10;
			for (int r = 0; r < reps; r++) md.fn<<<blocks, 256>>>( out, 0.999f, 0.001f, clk );
			hipEventRecord( e1 );
			hipEventSynchronize( e1 );
			float ms; hipEventElapsedTime( &ms, e0, e1 );
			std::vector<unsigned long long> h( blocks * 2 );
			hipMemcpy( h.data(), clk, blocks * 16, hipMemcpyDeviceToHost );
			std::vector<double> ghz;
			for (int i = 0; i < blocks; i++) ghz.push_back( (double)h[2 * i] / ((double)h[2 * i + 1] / 100e6) / 1e9 );
			std::sort( ghz.begin(), ghz.end() );
			const double clock = ghz[ghz.size() / 2];
			const double cyc = ms / reps * 1e-3 * clock * 1e9;
			if (md.insts)
			{
				const double insts = (double)blocks * 4 * ITERS * md.insts;          // wave64 VALU instructions per launch
				const double perSimd = insts / (cus * 4.0);
				printf( "{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, \"insts_per_iter\": %d, "
					"\"wave_insts_per_simd_per_cycle\": %.4f, \"cycles_per_wave_inst\": %.3f}\n",
					md.name, wavesPerSimd, ms / reps, clock, md.insts, perSimd / cyc, cyc / perSimd );
			}
			else
				printf( "{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, \"insts_per_iter\": null, "
					"\"blocks\": %d, \"iters\": %d, \"cycles_per_launch\": %.0f}\n", md.name, wavesPerSimd, ms / reps, clock, blocks, ITERS, cyc );
			hipEventDestroy( e0 ); hipEventDestroy( e1 );
			hipFree( out ); hipFree( clk );
		}
	}
	return 0;
}
