// VALU issue-rate probe (round 6): how many cycles one SIMD needs per wave64 VALU instruction, per
// instruction class, at 1 / 2 / 4 / 8 waves per SIMD.  This is the peak bench.py prices the traversal against.
//
// Method
//  * each lane runs 16 independent chains of one instruction class (an instruction's next use of its own result is 16
//    instructions later, beyond any VALU dependency latency), the loop body unrolled 4x: 64 VALU instructions per
//    iteration, exactly (the forms are pinned with inline asm; tools/valu_rate_isa.py counts them in the code object's
//    ISA and commits the loop bodies beside the results);
//  * every wave stamps s_memtime (shader-clock ticks, MI355X_MICROARCH.md "s_memtime tick = shader cycle") before and
//    after its loop, and records where it ran: HW_ID (SIMD, CU, SH, SE) and XCC_ID;
//  * per SIMD: cycles per instruction = (span of that SIMD's waves: last end - first start, in its own clock) /
//    (wave instructions the SIMD issued).  No clock frequency is assumed, and the waves' real placement is used
//    (not "4 waves per block land on 4 SIMDs"); the JSON line carries the median over SIMDs and the placement
//    histogram.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <vector>
#include <algorithm>

#define ITERS 1024
#define CHAINS 16
#define UNROLL 4
typedef float f2 __attribute__( (ext_vector_type( 2 )) );

struct WaveRec { unsigned long long t0, t1; unsigned hwid, xcc; };

__device__ inline void stamp_start( unsigned long long& t0 ) { t0 = __builtin_amdgcn_s_memtime(); }
__device__ inline void stamp_end( WaveRec* rec, unsigned long long t0 )
{
	const unsigned long long t1 = __builtin_amdgcn_s_memtime();
	unsigned hw, xcc;
	asm volatile( "s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"( hw ) );
	asm volatile( "s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"( xcc ) );
	const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	if ((threadIdx.x & 63) == 0) rec[wave] = { t0, t1, hw, xcc };   /* a vector store from lane 0 */
}

/* one instruction class: OP(x) is one VALU instruction on chain register x (a float VGPR, or a float2 pair for packed) */
#define DEFINE_PROBE( NAME, T, INIT, OP, FOLD )                                                         \
	__global__ __launch_bounds__( 256 ) void k_##NAME( float* out, float a, float b, WaveRec* rec )    \
	{                                                                                                   \
		const f2 a2 = { a, a }, b2 = { b, b };                                                          \
		const uint64_t m = 0x5555555555555555ull;                                                       \
		(void)a2; (void)b2; (void)m;                                                                    \
		T x[CHAINS];                                                                                    \
		for (int c = 0; c < CHAINS; c++) x[c] = INIT;                                                   \
		unsigned long long t0;                                                                          \
		stamp_start( t0 );                                                                              \
		for (int i = 0; i < ITERS; i++)                                                                 \
		{                                                                                               \
			_Pragma( "unroll" ) for (int u = 0; u < UNROLL; u++)                                        \
			{                                                                                           \
				OP( x[0] ); OP( x[1] ); OP( x[2] ); OP( x[3] ); OP( x[4] ); OP( x[5] ); OP( x[6] ); OP( x[7] ); \
				OP( x[8] ); OP( x[9] ); OP( x[10] ); OP( x[11] ); OP( x[12] ); OP( x[13] ); OP( x[14] ); OP( x[15] ); \
			}                                                                                           \
		}                                                                                               \
		stamp_end( rec, t0 );                                                                           \
		float s = 0;                                                                                    \
		for (int c = 0; c < CHAINS; c++) s += FOLD( x[c] );                                             \
		out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                                 \
	}

#define INITF ((float)threadIdx.x + (float)c)
#define INITP ((f2){ (float)threadIdx.x + (float)c, 1.0f })
#define FOLDF( v ) (v)
#define FOLDP( v ) ((v).x + (v).y)
#define OP_FMA( v ) asm volatile( "v_fma_f32 %0, %0, %1, %2" : "+v"( v ) : "v"( a ), "v"( b ) )
#define OP_ADD( v ) asm volatile( "v_add_f32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_MUL( v ) asm volatile( "v_mul_f32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_PKFMA( v ) asm volatile( "v_pk_fma_f32 %0, %0, %1, %2" : "+v"( v ) : "v"( a2 ), "v"( b2 ) )
#define OP_MAX3( v ) asm volatile( "v_max3_f32 %0, %0, %1, %2" : "+v"( v ) : "v"( a ), "v"( b ) )
#define OP_AND( v ) asm volatile( "v_and_b32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_ADDU( v ) asm volatile( "v_add_u32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_CVTB( v ) asm volatile( "v_cvt_f32_ubyte1 %0, %0" : "+v"( v ) )
#define OP_CND( v ) asm volatile( "v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"( v ) : "v"( a ), "s"( m ) )
#define OP_MOV( v ) asm volatile( "v_mov_b32 %0, %1" : "=v"( v ) : "v"( a ) )
#define OP_LDEXP( v ) asm volatile( "v_ldexp_f32 %0, %0, 1" : "+v"( v ) )
#define OP_RCP( v ) asm volatile( "v_rcp_f32 %0, %0" : "+v"( v ) )
/* the VOP2 / VOPC (32-bit encoded) forms of the classes above that were only probed as VOP3: an FMA accumulating into
   its destination, a select and a compare through VCC, a two-input max, a conversion */
#define OP_FMAC( v ) asm volatile( "v_fmac_f32_e32 %0, %1, %2" : "+v"( v ) : "v"( a ), "v"( b ) )
#define OP_CND32( v ) asm volatile( "v_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"( v ) : "v"( a ) )
#define OP_CMP32( v ) asm volatile( "v_cmp_lt_f32_e32 vcc, %0, %1" : : "v"( v ), "v"( a ) : "vcc" )
#define OP_MAX( v ) asm volatile( "v_max_f32_e32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_CVTU( v ) asm volatile( "v_cvt_f32_u32_e32 %0, %0" : "+v"( v ) )
/* round 6, second batch: the operations a node step could use instead of the 4-cycle ones above: integer max / min
   (ordered like the floats they hold when the floats are not negative), a byte select by SDWA (an OR with a magic
   exponent turns a node byte b into the float 2^23 + b), a float subtract, packed add / multiply, a shift, a bit-field
   extract, a byte permute, a median */
#define OP_MAXI( v ) asm volatile( "v_max_i32_e32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_MINU( v ) asm volatile( "v_min_u32_e32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_MAX3I( v ) asm volatile( "v_max3_i32 %0, %0, %1, %2" : "+v"( v ) : "v"( a ), "v"( b ) )
#define OP_ORSDWA( v ) asm volatile( "v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"( v ) : "v"( a ) )
#define OP_SUB( v ) asm volatile( "v_sub_f32_e32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
#define OP_PKADD( v ) asm volatile( "v_pk_add_f32 %0, %0, %1" : "+v"( v ) : "v"( a2 ) )
#define OP_PKMUL( v ) asm volatile( "v_pk_mul_f32 %0, %0, %1" : "+v"( v ) : "v"( a2 ) )
#define OP_SHR( v ) asm volatile( "v_lshrrev_b32_e32 %0, 3, %0" : "+v"( v ) )
#define OP_BFE( v ) asm volatile( "v_bfe_u32 %0, %0, 8, 8" : "+v"( v ) )
#define OP_PERM( v ) asm volatile( "v_perm_b32 %0, %0, %1, %2" : "+v"( v ) : "v"( a ), "v"( b ) )
#define OP_MED3( v ) asm volatile( "v_med3_f32 %0, %0, %1, %2" : "+v"( v ) : "v"( a ), "v"( b ) )
#define OP_CMPI( v ) asm volatile( "v_cmp_lt_i32_e32 vcc, %0, %1" : : "v"( v ), "v"( a ) : "vcc" )
#define OP_MINF( v ) asm volatile( "v_min_f32_e32 %0, %0, %1" : "+v"( v ) : "v"( a ) )
/* a compare writing an SGPR pair: the chain register is only read (no VALU result to wait on) */
#define OP_CMP( v ) do { uint64_t sdst; asm volatile( "v_cmp_lt_f32_e64 %0, %1, %2" : "=s"( sdst ) : "v"( v ), "v"( a ) ); } while (0)

DEFINE_PROBE( fma, float, INITF, OP_FMA, FOLDF )
DEFINE_PROBE( add, float, INITF, OP_ADD, FOLDF )
DEFINE_PROBE( mul, float, INITF, OP_MUL, FOLDF )
DEFINE_PROBE( pkfma, f2, INITP, OP_PKFMA, FOLDP )
DEFINE_PROBE( max3, float, INITF, OP_MAX3, FOLDF )
DEFINE_PROBE( and, float, INITF, OP_AND, FOLDF )
DEFINE_PROBE( addu, float, INITF, OP_ADDU, FOLDF )
DEFINE_PROBE( cvtb, float, INITF, OP_CVTB, FOLDF )
DEFINE_PROBE( cnd, float, INITF, OP_CND, FOLDF )
DEFINE_PROBE( mov, float, INITF, OP_MOV, FOLDF )
DEFINE_PROBE( ldexp, float, INITF, OP_LDEXP, FOLDF )
DEFINE_PROBE( rcp, float, INITF, OP_RCP, FOLDF )
DEFINE_PROBE( cmp, float, INITF, OP_CMP, FOLDF )
DEFINE_PROBE( fmac, float, INITF, OP_FMAC, FOLDF )
DEFINE_PROBE( cnd32, float, INITF, OP_CND32, FOLDF )
DEFINE_PROBE( cmp32, float, INITF, OP_CMP32, FOLDF )
DEFINE_PROBE( max, float, INITF, OP_MAX, FOLDF )
DEFINE_PROBE( cvtu, float, INITF, OP_CVTU, FOLDF )
DEFINE_PROBE( maxi, float, INITF, OP_MAXI, FOLDF )
DEFINE_PROBE( minu, float, INITF, OP_MINU, FOLDF )
DEFINE_PROBE( max3i, float, INITF, OP_MAX3I, FOLDF )
DEFINE_PROBE( orsdwa, float, INITF, OP_ORSDWA, FOLDF )
DEFINE_PROBE( sub, float, INITF, OP_SUB, FOLDF )
DEFINE_PROBE( pkadd, f2, INITP, OP_PKADD, FOLDP )
DEFINE_PROBE( pkmul, f2, INITP, OP_PKMUL, FOLDP )
DEFINE_PROBE( shr, float, INITF, OP_SHR, FOLDF )
DEFINE_PROBE( bfe, float, INITF, OP_BFE, FOLDF )
DEFINE_PROBE( perm, float, INITF, OP_PERM, FOLDF )
DEFINE_PROBE( med3, float, INITF, OP_MED3, FOLDF )
DEFINE_PROBE( cmpi, float, INITF, OP_CMPI, FOLDF )
DEFINE_PROBE( minf, float, INITF, OP_MINF, FOLDF )

/* the BVH4 node step's mix, compiler-scheduled (round 3's probe): two packed slab-plane FMAs, an entry max3 and an exit
   min3, the padded exit, two compares and a select into an integer sort key, an unsigned compare-exchange; 8 chains.
   Its VALU count per iteration is read from the ISA (tools/valu_rate_isa.py), not assumed */
__global__ __launch_bounds__( 256 ) void k_mix( float* out, float a, float b, WaveRec* rec )
{
	const f2 a2 = { a, a }, b2 = { b, -b };
	f2 p[8];
	float m[8];
	uint32_t lo[8], hi[8];
	for (int c = 0; c < 8; c++) p[c] = (f2){ (float)threadIdx.x + c, (float)c }, m[c] = 0.5f * c, lo[c] = 0xffffffffu, hi[c] = 0;
	unsigned long long t0;
	stamp_start( t0 );
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
	stamp_end( rec, t0 );
	float s = 0;
	for (int c = 0; c < 8; c++) s += p[c].x + p[c].y + m[c] + (float)(lo[c] ^ hi[c]);
	out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*KernelFn)( float*, float, float, WaveRec* );

int main( int argc, char** argv )
{
	/* --mode NAME: that class only; --waves W: that occupancy only (the counter passes, tools/valu_rate_pmc.sh) */
	const char* only = nullptr;
	int onlyWaves = 0;
	for (int i = 1; i + 1 < argc; i += 2)
		if (!strcmp( argv[i], "--mode" )) only = argv[i + 1];
		else if (!strcmp( argv[i], "--waves" )) onlyWaves = atoi( argv[i + 1] );
	hipDeviceProp_t p;
	hipGetDeviceProperties( &p, 0 );
	const int cus = p.multiProcessorCount;
	/* insts: VALU instructions per loop iteration (64 for the pinned classes; the mix's from the ISA, 0 here) */
	struct { const char* name; KernelFn fn; int insts; } modes[] = {
		{ "fma", k_fma, 64 }, { "add", k_add, 64 }, { "mul", k_mul, 64 }, { "pkfma", k_pkfma, 64 }, { "max3", k_max3, 64 },
		{ "and", k_and, 64 }, { "addu", k_addu, 64 }, { "cvtb", k_cvtb, 64 }, { "cnd", k_cnd, 64 }, { "mov", k_mov, 64 },
		{ "ldexp", k_ldexp, 64 }, { "rcp", k_rcp, 64 }, { "cmp", k_cmp, 64 }, { "fmac", k_fmac, 64 }, { "cnd32", k_cnd32, 64 },
		{ "cmp32", k_cmp32, 64 }, { "max", k_max, 64 }, { "cvtu", k_cvtu, 64 }, { "mix", k_mix, 0 },
		{ "maxi", k_maxi, 64 }, { "minu", k_minu, 64 }, { "max3i", k_max3i, 64 }, { "orsdwa", k_orsdwa, 64 }, { "sub", k_sub, 64 },
		{ "pkadd", k_pkadd, 64 }, { "pkmul", k_pkmul, 64 }, { "shr", k_shr, 64 }, { "bfe", k_bfe, 64 }, { "perm", k_perm, 64 },
		{ "med3", k_med3, 64 }, { "cmpi", k_cmpi, 64 }, { "minf", k_minf, 64 } };
	for (auto& md : modes)
	{
		if (only && strcmp( only, md.name )) continue;
		for (int wavesPerSimd : { 1, 2, 4, 8 })
		{
			if (onlyWaves && wavesPerSimd != onlyWaves) continue;
			const int blocks = cus * wavesPerSimd;   // 4 waves per block
			const int waves = blocks * 4;
			float* out; WaveRec* rec;
			hipMalloc( &out, (size_t)blocks * 256 * 4 );
			hipMalloc( &rec, (size_t)waves * sizeof( WaveRec ) );
			md.fn<<<blocks, 256>>>( out, 0.999f, 0.001f, rec );   /* warm-up (clocks up, code loaded) */
			hipEvent_t e0, e1;
			hipEventCreate( &e0 ); hipEventCreate( &e1 );
			hipEventRecord( e0 );
			md.fn<<<blocks, 256>>>( out, 0.999f, 0.001f, rec );
			hipEventRecord( e1 );
			hipEventSynchronize( e1 );
			float ms; hipEventElapsedTime( &ms, e0, e1 );
			std::vector<WaveRec> h( waves );
			hipMemcpy( h.data(), rec, waves * sizeof( WaveRec ), hipMemcpyDeviceToHost );
			/* per SIMD: key = XCC, SE / SH / CU (HW_ID[15:8]), SIMD (HW_ID[5:4]) */
			struct Simd { unsigned long long lo = ~0ull, hi = 0; int waves = 0; };
			std::map<unsigned, Simd> simds;
			for (const WaveRec& r : h)
			{
				const unsigned key = (r.xcc & 0xf) << 16 | (r.hwid & 0xff00u) | ((r.hwid >> 4) & 3u);
				Simd& s = simds[key];
				s.lo = std::min( s.lo, r.t0 ), s.hi = std::max( s.hi, r.t1 ), s.waves++;
			}
			std::map<int, int> hist;   /* waves per SIMD -> SIMDs */
			for (auto& kv : simds) hist[kv.second.waves]++;
			printf( "{\"mode\": \"%s\", \"waves_per_simd\": %d, \"blocks\": %d, \"iters\": %d, \"chains\": %d, \"launch_ms\": %.4f, "
				"\"simds\": %zu, \"placement\": {", md.name, wavesPerSimd, blocks, ITERS, CHAINS, ms, simds.size() );
			bool first = true;
			for (auto& kv : hist) printf( "%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second ), first = false;
			printf( "}" );
			/* cycles per wave instruction on each SIMD: its span over the instructions its waves issued */
			std::vector<double> cpi, span;
			for (auto& kv : simds)
			{
				const double cyc = (double)(kv.second.hi - kv.second.lo);
				span.push_back( cyc );
				if (md.insts) cpi.push_back( cyc / ((double)kv.second.waves * ITERS * md.insts) );
				else cpi.push_back( cyc / ((double)kv.second.waves * ITERS) );   /* per iteration: divided by the ISA count later */
			}
			std::sort( cpi.begin(), cpi.end() ), std::sort( span.begin(), span.end() );
			const double med = cpi[cpi.size() / 2], p10 = cpi[cpi.size() / 10], p90 = cpi[cpi.size() * 9 / 10];
			const double clockGhz = span.back() / (ms * 1e-3) / 1e9;   /* the slowest SIMD's span over the launch: a lower bound of the clock */
			if (md.insts)
				printf( ", \"insts_per_iter\": %d, \"cycles_per_wave_inst\": %.3f, \"p10\": %.3f, \"p90\": %.3f", md.insts, med, p10, p90 );
			else
				printf( ", \"insts_per_iter\": null, \"cycles_per_iter\": %.2f, \"p10\": %.2f, \"p90\": %.2f", med, p10, p90 );
			printf( ", \"span_cycles_max\": %.0f, \"clock_lower_bound_ghz\": %.3f}\n", span.back(), clockGhz );
			fflush( stdout );
			hipEventDestroy( e0 ); hipEventDestroy( e1 );
			hipFree( out ); hipFree( rec );
		}
	}
	return 0;
}
