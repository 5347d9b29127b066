/* bvh_gpu.hip - GPU BVH2 construction (PLOC + SAH leaf collapse), see bvh_gpu.h.

   Layout produced (lh2_device.h): 64-B child-pair nodes in depth-first pre-order, so descending
   always increases the node index (the traversal's termination argument), and 48-B triangles
   (v0, origIdx)(e1)(e2) in leaf order, e1/e2 computed in fp32 exactly as bvh_build.cpp does. */
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "bvh_gpu.h"
#include "lh2_device.h"
#include "lh2_kernels.h"

namespace lh2 {
void FatalError( const char* fmt, ... );
}

#define CHK( stmt ) do { hipError_t e_ = (stmt); if (e_ != hipSuccess) lh2::FatalError( "%s failed: %s (%s:%d)", #stmt, hipGetErrorString( e_ ), __FILE__, __LINE__ ); } while (0)

namespace {

struct alignas( 16 ) Box8 { float4 lo, hi; };
using lh2::GpuTlasArgs;

constexpr float INF = __builtin_huge_valf();

__device__ __forceinline__ Box8 box_union( const Box8& a, const Box8& b )
{
	Box8 r;
	r.lo = make_float4( fminf( a.lo.x, b.lo.x ), fminf( a.lo.y, b.lo.y ), fminf( a.lo.z, b.lo.z ), 0 );
	r.hi = make_float4( fmaxf( a.hi.x, b.hi.x ), fmaxf( a.hi.y, b.hi.y ), fmaxf( a.hi.z, b.hi.z ), 0 );
	return r;
}
/* surface area; NaN (boxes of empty instances) counts as infinite */
__device__ __forceinline__ float box_area( const Box8& b )
{
	const float dx = b.hi.x - b.lo.x, dy = b.hi.y - b.lo.y, dz = b.hi.z - b.lo.z;
	const float a = 2.0f * (dx * dy + dx * dz + dy * dz);
	return a == a ? fmaxf( a, 0.0f ) : INF;
}

/* order-preserving float <-> uint for atomicMin / atomicMax */
__device__ __forceinline__ uint32_t f2o( float f ) { const uint32_t u = __float_as_uint( f ); return (u & 0x80000000u) ? ~u : (u | 0x80000000u); }
__host__ __device__ __forceinline__ float o2f( uint32_t o ) { const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o; float f; memcpy( &f, &u, 4 ); return f; }

__device__ __forceinline__ uint64_t expand21( uint32_t v )
{
	uint64_t x = v & 0x1fffffu;
	x = (x | x << 32) & 0x1f00000000ffffull;
	x = (x | x << 16) & 0x1f0000ff0000ffull;
	x = (x | x << 8) & 0x100f00f00f00f00full;
	x = (x | x << 4) & 0x10c30c30c30c30c3ull;
	x = (x | x << 2) & 0x1249249249249249ull;
	return x;
}
__device__ __forceinline__ uint32_t quant( float c, float lo, float scale, float maxq )
{
	const float q = (c - lo) * scale;
	return (uint32_t)fminf( fmaxf( q == q ? q : 0.0f, 0.0f ), maxq );
}

/* ---- wave / block reductions of 12 bound values (centroid lo/hi, geometry lo/hi) ---------- */
__device__ __forceinline__ void reduce_bounds( float v[12], uint32_t* red )
{
	for (int off = 32; off > 0; off >>= 1)
		for (int k = 0; k < 12; k++)
		{
			const float o = __shfl_xor( v[k], off );
			v[k] = ((k / 3) & 1) ? fmaxf( v[k], o ) : fminf( v[k], o );
		}
	if ((threadIdx.x & 63) == 0)
		for (int k = 0; k < 12; k++)
			if (v[k] == v[k] && v[k] != INF && v[k] != -INF)
			{
				if ((k / 3) & 1) atomicMax( red + k, f2o( v[k] ) ); else atomicMin( red + k, f2o( v[k] ) );
			}
}
__device__ __forceinline__ void grow_bounds( float v[12], const Box8& b )
{
	if (!(b.lo.x == b.lo.x)) return;   /* NaN box: empty instance */
	const float c[3] = { 0.5f * b.lo.x + 0.5f * b.hi.x, 0.5f * b.lo.y + 0.5f * b.hi.y, 0.5f * b.lo.z + 0.5f * b.hi.z };
	const float lo[3] = { b.lo.x, b.lo.y, b.lo.z }, hi[3] = { b.hi.x, b.hi.y, b.hi.z };
	for (int k = 0; k < 3; k++)
		v[k] = fminf( v[k], c[k] ), v[3 + k] = fmaxf( v[3 + k], c[k] ), v[6 + k] = fminf( v[6 + k], lo[k] ), v[9 + k] = fmaxf( v[9 + k], hi[k] );
}
__device__ __forceinline__ void init_bounds( float v[12] )
{
	for (int k = 0; k < 12; k++) v[k] = ((k / 3) & 1) ? -INF : INF;
}

/* the largest grid exponent of a quantized node (box4q scales the ray's clamped reciprocal +-1e30 by 2^e: 1e30 * 2^27
   stays finite) */
#define LH2_QEXP_MAX 27

__global__ void k_reset_red( uint32_t* red )
{
	const int k = threadIdx.x;
	if (k < 12) red[k] = ((k / 3) & 1) ? 0u : 0xffffffffu;
	else if (k < 16) red[k] = 0;
}

/* triangle boxes from the CoreTri records (vertex0..2 = float4 8..10 of 11) */
__global__ __launch_bounds__( 256 ) void k_tri_bounds( const float4* __restrict__ tris, int n, Box8* __restrict__ pb, uint32_t* red )
{
	float v[12];
	init_bounds( v );
	for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
	{
		const float4 a = tris[(size_t)i * 11 + 8], b = tris[(size_t)i * 11 + 9], c = tris[(size_t)i * 11 + 10];
		Box8 bx;
		bx.lo = make_float4( fminf( fminf( a.x, b.x ), c.x ), fminf( fminf( a.y, b.y ), c.y ), fminf( fminf( a.z, b.z ), c.z ), 0 );
		bx.hi = make_float4( fmaxf( fmaxf( a.x, b.x ), c.x ), fmaxf( fmaxf( a.y, b.y ), c.y ), fmaxf( fmaxf( a.z, b.z ), c.z ), 0 );
		pb[i] = bx;
		grow_bounds( v, bx );
	}
	reduce_bounds( v, red );
}

/* world box of one instance: the 8 transformed corners of its mesh bounds, padded by a relative
   epsilon (the ray is transformed in fp32 on the device); same rule as the host TLAS build */
__device__ Box8 instance_box( const float* __restrict__ T, const float* __restrict__ mb )
{
	Box8 b;
	const float nanv = __builtin_nanf( "" );
	if (!(mb[0] <= mb[3]))
	{
		b.lo = make_float4( nanv, nanv, nanv, 0 ), b.hi = b.lo;
		return b;
	}
	float lo[3] = { 1e30f, 1e30f, 1e30f }, hi[3] = { -1e30f, -1e30f, -1e30f };
	for (int c = 0; c < 8; c++)
	{
		const float p[3] = { (c & 1) ? mb[3] : mb[0], (c & 2) ? mb[4] : mb[1], (c & 4) ? mb[5] : mb[2] };
		for (int k = 0; k < 3; k++)
		{
			const float* r = T + k * 4;
			const float v = r[0] * p[0] + r[1] * p[1] + r[2] * p[2] + r[3];
			lo[k] = fminf( lo[k], v ), hi[k] = fmaxf( hi[k], v );
		}
	}
	for (int k = 0; k < 3; k++)
	{
		const float e = 1e-5f * fmaxf( fabsf( lo[k] ), fabsf( hi[k] ) ) + 1e-30f;
		lo[k] -= e, hi[k] += e;
	}
	b.lo = make_float4( lo[0], lo[1], lo[2], 0 ), b.hi = make_float4( hi[0], hi[1], hi[2], 0 );
	return b;
}

__global__ __launch_bounds__( 256 ) void k_inst_bounds( const float* __restrict__ T, const int* __restrict__ mesh, const float* __restrict__ mb,
	int n, Box8* __restrict__ pb, uint32_t* red )
{
	float v[12];
	init_bounds( v );
	for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
	{
		const Box8 bx = instance_box( T + (size_t)i * 16, mb + (size_t)mesh[i] * 6 );
		pb[i] = bx;
		grow_bounds( v, bx );
	}
	reduce_bounds( v, red );
}

__global__ __launch_bounds__( 256 ) void k_morton( const Box8* __restrict__ pb, int n, const uint32_t* __restrict__ red, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n) return;
	float lo[3], sc[3];
	for (int k = 0; k < 3; k++)
	{
		lo[k] = o2f( red[k] );
		const float ext = o2f( red[3 + k] ) - lo[k];
		sc[k] = ext > 0 ? 2097152.0f / ext : 0.0f;
	}
	const Box8 b = pb[i];
	const float c[3] = { 0.5f * b.lo.x + 0.5f * b.hi.x, 0.5f * b.lo.y + 0.5f * b.hi.y, 0.5f * b.lo.z + 0.5f * b.hi.z };
	uint64_t m = 0;
	for (int k = 0; k < 3; k++) m |= expand21( quant( c[k], lo[k], sc[k], 2097151.0f ) ) << (2 - k);
	keys[i] = m, vals[i] = (uint32_t)i;
}

/* leaves in Morton order: node k = sorted position k */
__global__ __launch_bounds__( 256 ) void k_init_leaves( const uint32_t* __restrict__ vals, const Box8* __restrict__ pb, int n, Box8* __restrict__ boxes,
	uint32_t* __restrict__ P, uint32_t* __restrict__ I, float* __restrict__ cost, int* __restrict__ parent, uint32_t* __restrict__ leafOrig,
	int* __restrict__ clNode, Box8* __restrict__ clBox )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n) return;
	const uint32_t o = vals[i];
	const Box8 b = pb[o];
	boxes[i] = b, P[i] = 1, I[i] = 0, cost[i] = box_area( b ), parent[i] = -1, leafOrig[i] = o;
	clNode[i] = i, clBox[i] = b;
}

/* nearest neighbour of cluster i within +-r by merged surface area.  Pairs are ordered by (area,
   index gap, odd lower index, lower index): one total order, so the best pair overall is mutual and
   every round merges; the gap / parity keys pair up equal boxes as (2k, 2k+1), so identical
   primitives give a balanced tree instead of a chain */
__device__ __forceinline__ bool pair_better( float d, int i, int j, float bd, int bj )
{
	if (d != bd) return d < bd;
	const int g = abs( i - j ), bg = abs( i - bj );
	if (g != bg) return g < bg;
	const int m = min( i, j ), bm = min( i, bj );
	if ((m & 1) != (bm & 1)) return (m & 1) == 0;
	return m < bm;
}
__device__ __forceinline__ int nearest( const Box8* __restrict__ cb, int i, int n, int r, const Box8& bi )
{
	float best = INF;
	int bj = -1;
	const int j0 = max( 0, i - r ), j1 = min( n - 1, i + r );
	for (int j = j0; j <= j1; j++)
	{
		if (j == i) continue;
		const float d = box_area( box_union( bi, cb[j] ) );
		if (bj < 0 || pair_better( d, i, j, best, bj )) best = d, bj = j;
	}
	return bj;
}

__global__ __launch_bounds__( 256 ) void k_nn( const Box8* __restrict__ cb, int n, int r, int* __restrict__ nn )
{
	__shared__ Box8 tile[256 + 64];
	const int s = blockIdx.x * 256, t0 = s - r, cnt = min( n, s + 256 + r ) - max( 0, t0 );
	for (int k = threadIdx.x; k < 256 + 2 * r; k += 256)
	{
		const int j = t0 + k;
		if (j >= 0 && j < n) tile[k] = cb[j];
	}
	(void)cnt;
	__syncthreads();
	const int i = s + threadIdx.x;
	if (i >= n) return;
	const Box8 bi = tile[i - t0];
	float best = INF;
	int bj = -1;
	const int j0 = max( 0, i - r ), j1 = min( n - 1, i + r );
	for (int j = j0; j <= j1; j++)
	{
		if (j == i) continue;
		const float d = box_area( box_union( bi, tile[j - t0] ) );
		if (bj < 0 || pair_better( d, i, j, best, bj )) best = d, bj = j;
	}
	nn[i] = bj;
}

__global__ __launch_bounds__( 256 ) void k_flags( const int* __restrict__ nn, int n, uint64_t* __restrict__ flags )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n) return;
	const int j = nn[i];
	const bool mutual = j >= 0 && nn[j] == i;
	const uint64_t keep = (mutual && j < i) ? 0u : 1u, made = (mutual && i < j) ? 1u : 0u;
	flags[i] = keep | (made << 32);
}

/* create the node of a mutual pair (i < j): SAH cost and leaf collapse decided here, the children
   being complete already */
__device__ __forceinline__ void make_node( int id, int a, int b, const Box8& box, bool root, int maxLeaf, float ct,
	Box8* boxes, int* child, int* parent, uint32_t* P, uint32_t* I, float* cost )
{
	const float A = box_area( box );
	const uint32_t p = P[a] + P[b];
	const float split = ct * A + cost[a] + cost[b];
	const float leaf = (float)p * A;
	uint32_t in;
	float c;
	if (!root && (int)p <= maxLeaf && leaf <= split) in = 0, c = leaf;
	else in = 1 + I[a] + I[b], c = split;
	boxes[id] = box;
	((int2*)child)[id] = make_int2( a, b );
	parent[id] = -1, parent[a] = id, parent[b] = id;
	P[id] = p, I[id] = in, cost[id] = c;
}

__global__ __launch_bounds__( 256 ) void k_merge( const int* __restrict__ clNodeIn, const Box8* __restrict__ clBoxIn, const int* __restrict__ nn,
	const uint64_t* __restrict__ flags, const uint64_t* __restrict__ scan, int n, int nodeBase, int maxLeaf, float ct,
	int* __restrict__ clNodeOut, Box8* __restrict__ clBoxOut, Box8* boxes, int* child, int* parent, uint32_t* P, uint32_t* I, float* cost, uint32_t* red )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n) return;
	const uint64_t f = flags[i], s = scan[i];
	if (i == n - 1)
	{
		red[12] = (uint32_t)(s & 0xffffffffu) + (uint32_t)(f & 0xffffffffu);
		red[13] = (uint32_t)(s >> 32) + (uint32_t)(f >> 32);
	}
	if (!(f & 1)) return;
	const uint32_t pos = (uint32_t)(s & 0xffffffffu);
	if (f >> 32)
	{
		const int j = nn[i];
		const int id = nodeBase + (int)(s >> 32);
		const Box8 b = box_union( clBoxIn[i], clBoxIn[j] );
		make_node( id, clNodeIn[i], clNodeIn[j], b, n == 2, maxLeaf, ct, boxes, child, parent, P, I, cost );
		clNodeOut[pos] = id, clBoxOut[pos] = b;
	}
	else clNodeOut[pos] = clNodeIn[i], clBoxOut[pos] = clBoxIn[i];
}

/* ---- emission: walk up to the root summing left-sibling interior nodes / primitives ---------- */
__device__ __forceinline__ void emit_node( int x, int N, int tlas, int nodeBase, uint32_t triBase, const Box8* __restrict__ boxes, const int* __restrict__ child,
	const int* __restrict__ parent, const uint32_t* __restrict__ P, const uint32_t* __restrict__ I, const uint32_t* __restrict__ leafOrig,
	const float4* __restrict__ coreTris, float4* __restrict__ nodes, float4* __restrict__ tris, uint32_t* depthMax )
{
	int pre = 0, depth = 1, c = x;
	uint32_t off = 0;
	bool hidden = false;
	for (int p = parent[c]; p >= 0; c = p, p = parent[c])
	{
		if (I[p] == 0) hidden = true;
		const int2 ch = ((const int2*)child)[p];
		if (ch.y == c) pre += 1 + (int)I[ch.x], off += P[ch.x];
		else pre += 1;
		depth++;
	}
	if (x < N && !tlas)
	{
		const uint32_t o = leafOrig[x];
		const float4 a = coreTris[(size_t)o * 11 + 8], b = coreTris[(size_t)o * 11 + 9], cc = coreTris[(size_t)o * 11 + 10];
		float4* t = tris + (size_t)(triBase + off) * 3;
		t[0] = make_float4( a.x, a.y, a.z, __uint_as_float( o ) );
		t[1] = make_float4( b.x - a.x, b.y - a.y, b.z - a.z, 0 );
		t[2] = make_float4( cc.x - a.x, cc.y - a.y, cc.z - a.z, 0 );
	}
	if (hidden || I[x] == 0) return;
	const int2 ch = ((const int2*)child)[x];
	const Box8 A = boxes[ch.x], B = boxes[ch.y];
	int ra, rb;
	if (I[ch.x] > 0) ra = nodeBase + pre + 1;
	else ra = tlas ? MAKE_LEAF( leafOrig[ch.x], 1 ) : MAKE_LEAF( triBase + off, P[ch.x] );
	if (I[ch.y] > 0) rb = nodeBase + pre + 1 + (int)I[ch.x];
	else rb = tlas ? MAKE_LEAF( leafOrig[ch.y], 1 ) : MAKE_LEAF( triBase + off + P[ch.x], P[ch.y] );
	float4* o = nodes + (size_t)(nodeBase + pre) * 4;
	o[0] = make_float4( A.lo.x, A.hi.x, A.lo.y, A.hi.y );
	o[1] = make_float4( B.lo.x, B.hi.x, B.lo.y, B.hi.y );
	o[2] = make_float4( A.lo.z, A.hi.z, B.lo.z, B.hi.z );
	o[3] = make_float4( __int_as_float( ra ), __int_as_float( rb ), 0, 0 );
	atomicMax( depthMax, (uint32_t)depth );
}

__global__ __launch_bounds__( 256 ) void k_emit( int N, int tlas, int nodeBase, uint32_t triBase, const Box8* __restrict__ boxes, const int* __restrict__ child,
	const int* __restrict__ parent, const uint32_t* __restrict__ P, const uint32_t* __restrict__ I, const uint32_t* __restrict__ leafOrig,
	const float4* __restrict__ coreTris, float4* __restrict__ nodes, float4* __restrict__ tris, uint32_t* red )
{
	const int x = blockIdx.x * 256 + threadIdx.x;
	if (x >= 2 * N - 1) return;
	emit_node( x, N, tlas, nodeBase, triBase, boxes, child, parent, P, I, leafOrig, coreTris, nodes, tris, red + 14 );
}

__global__ void k_tlas_check( const uint32_t* red, int maxBlasDepth, int tlasFactor, int* sceneError, int* tlasDepth )
{
	const int d = (int)red[14];
	*tlasDepth = d;
	if (tlasFactor * d + maxBlasDepth >= LH2_STACK_TOTAL - 1) atomicOr( sceneError, LH2_SCENE_ERR_DEPTH );
}

/* ---- single-workgroup TLAS build (count <= LH2_TLAS_WG_MAX): no host round trip ---------- */
struct TlasScratch
{
	Box8* prim; Box8* boxes; Box8* cl0; Box8* cl1; int* clNode0; int* clNode1;
	int* child; int* parent; uint32_t* P; uint32_t* I; float* cost; uint32_t* leafOrig; int* nn;
};

/* exclusive scan of f[0..n) in place (n <= 4 x 1024), all 1024 threads */
__device__ uint32_t block_scan4( uint32_t* f, int n, uint32_t* wt )
{
	const int t = threadIdx.x, lane = t & 63;
	uint32_t v[4], s = 0;
	for (int k = 0; k < 4; k++) { const int idx = 4 * t + k; v[k] = idx < n ? f[idx] : 0u; s += v[k]; }
	uint32_t x = s;
	for (int off = 1; off < 64; off <<= 1) { const uint32_t y = __shfl_up( x, off ); if (lane >= off) x += y; }
	if (lane == 63) wt[t >> 6] = x;
	__syncthreads();
	if (t == 0) { uint32_t acc = 0; for (int w = 0; w < 16; w++) { const uint32_t q = wt[w]; wt[w] = acc; acc += q; } wt[16] = acc; }
	__syncthreads();
	uint32_t e = wt[t >> 6] + x - s;
	for (int k = 0; k < 4; k++) { const int idx = 4 * t + k; if (idx < n) f[idx] = e; e += v[k]; }
	const uint32_t total = wt[16];
	__syncthreads();
	return total;
}

__global__ __launch_bounds__( 1024 ) void k_tlas_build_wg( const GpuTlasArgs a, const TlasScratch s, int radius )
{
	__shared__ uint64_t keys[LH2_TLAS_WG_MAX];
	__shared__ uint32_t f[LH2_TLAS_WG_MAX];
	__shared__ float redf[16][6];
	__shared__ uint32_t wt[17];
	__shared__ uint32_t depthMax;
	const int N = a.count, t = threadIdx.x;
	/* A: instance world boxes + centroid bounds */
	float v[12];
	init_bounds( v );
	for (int i = t; i < N; i += 1024)
	{
		const Box8 bx = instance_box( a.T + (size_t)i * 16, a.meshBounds + (size_t)a.instMesh[i] * 6 );
		s.prim[i] = bx;
		grow_bounds( v, bx );
	}
	for (int off = 32; off > 0; off >>= 1)
		for (int k = 0; k < 6; k++) { const float o = __shfl_xor( v[k], off ); v[k] = k >= 3 ? fmaxf( v[k], o ) : fminf( v[k], o ); }
	if ((t & 63) == 0) for (int k = 0; k < 6; k++) redf[t >> 6][k] = v[k];
	if (t == 0) depthMax = 0;
	__syncthreads();
	float lo[3], sc[3];
	for (int k = 0; k < 3; k++)
	{
		float l = INF, h = -INF;
		for (int w = 0; w < 16; w++) l = fminf( l, redf[w][k] ), h = fmaxf( h, redf[w][3 + k] );
		lo[k] = l;
		sc[k] = (h - l) > 0 ? 1024.0f / (h - l) : 0.0f;
	}
	/* B: 30-bit Morton keys, bitonic sort in LDS */
	int P2 = 1;
	while (P2 < N) P2 <<= 1;
	for (int i = t; i < P2; i += 1024)
	{
		uint64_t key = ~0ull;
		if (i < N)
		{
			const Box8 b = s.prim[i];
			const float c[3] = { 0.5f * b.lo.x + 0.5f * b.hi.x, 0.5f * b.lo.y + 0.5f * b.hi.y, 0.5f * b.lo.z + 0.5f * b.hi.z };
			uint64_t m = 0;
			for (int k = 0; k < 3; k++) m |= expand21( quant( c[k], lo[k], sc[k], 1023.0f ) ) << (2 - k);
			key = (m << 32) | (uint32_t)i;
		}
		keys[i] = key;
	}
	__syncthreads();
	for (int k = 2; k <= P2; k <<= 1)
		for (int j = k >> 1; j > 0; j >>= 1)
		{
			for (int i = t; i < P2; i += 1024)
			{
				const int ixj = i ^ j;
				if (ixj > i)
				{
					const uint64_t x = keys[i], y = keys[ixj];
					if (((i & k) == 0) == (x > y)) keys[i] = y, keys[ixj] = x;
				}
			}
			__syncthreads();
		}
	/* C: leaves */
	for (int i = t; i < N; i += 1024)
	{
		const uint32_t o = (uint32_t)(keys[i] & 0xffffffffu);
		const Box8 b = s.prim[o];
		s.boxes[i] = b, s.P[i] = 1, s.I[i] = 0, s.cost[i] = 0, s.parent[i] = -1, s.leafOrig[i] = o;
		s.clNode0[i] = i, s.cl0[i] = b;
	}
	__syncthreads();
	/* D: PLOC rounds */
	int n = N, made = 0, cur = 0;
	while (n > 1)
	{
		const Box8* cb = cur ? s.cl1 : s.cl0;
		const int* cn = cur ? s.clNode1 : s.clNode0;
		Box8* ob = cur ? s.cl0 : s.cl1;
		int* on = cur ? s.clNode0 : s.clNode1;
		for (int i = t; i < n; i += 1024) s.nn[i] = nearest( cb, i, n, radius, cb[i] );
		__syncthreads();
		for (int i = t; i < n; i += 1024)
		{
			const int j = s.nn[i];
			const bool mutual = j >= 0 && s.nn[j] == i;
			f[i] = ((mutual && j < i) ? 0u : 1u) | ((mutual && i < j) ? 0x10000u : 0u);
		}
		__syncthreads();
		uint32_t fl[4];
		for (int k = 0; k < 4; k++) { const int idx = 4 * t + k; fl[k] = idx < n ? f[idx] : 0u; }
		const uint32_t total = block_scan4( f, n, wt );
		for (int k = 0; k < 4; k++)
		{
			const int i = 4 * t + k;
			if (i >= n || !(fl[k] & 1u)) continue;
			const uint32_t pos = f[i] & 0xffffu;
			if (fl[k] >> 16)
			{
				const int j = s.nn[i];
				const int id = N + made + (int)(f[i] >> 16);
				const Box8 b = box_union( cb[i], cb[j] );
				make_node( id, cn[i], cn[j], b, true, 1, 1.0f, s.boxes, s.child, s.parent, s.P, s.I, s.cost );
				on[pos] = id, ob[pos] = b;
			}
			else on[pos] = cn[i], ob[pos] = cb[i];
		}
		__syncthreads();
		n = (int)(total & 0xffffu), made += (int)(total >> 16), cur ^= 1;
	}
	/* E: emission (all nodes interior: one instance per leaf) */
	uint32_t dm = 0;
	for (int x = t; x < 2 * N - 1; x += 1024)
		emit_node( x, N, 1, a.nodeBase, 0, s.boxes, s.child, s.parent, s.P, s.I, s.leafOrig, nullptr, a.nodes, nullptr, &depthMax );
	(void)dm;
	__syncthreads();
	if (t == 0)
	{
		*a.tlasDepth = (int)depthMax;
		if (a.tlasFactor * (int)depthMax + a.maxBlasDepth >= LH2_STACK_TOTAL - 1) atomicOr( a.sceneError, LH2_SCENE_ERR_DEPTH );
	}
}

__global__ __launch_bounds__( 256 ) void k_relocate( const float4* __restrict__ src, int count, int nodeBase, uint32_t triBase, float4* __restrict__ dst )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= count) return;
	const float4* s = src + (size_t)i * 4;
	float4* d = dst + (size_t)(nodeBase + i) * 4;
	d[0] = s[0], d[1] = s[1], d[2] = s[2];
	const float4 r = s[3];
	int ref[2] = { __float_as_int( r.x ), __float_as_int( r.y ) };
	for (int c = 0; c < 2; c++) ref[c] = ref[c] >= 0 ? ref[c] + nodeBase : MAKE_LEAF( LEAF_FIRST( ref[c] ) + triBase, LEAF_COUNT( ref[c] ) );
	d[3] = make_float4( __int_as_float( ref[0] ), __int_as_float( ref[1] ), 0, 0 );
}

/* BVH4 relocation: interior references + nodeBase, leaf triangle ranges + triBase */
__global__ __launch_bounds__( 256 ) void k_relocate4( const float4* __restrict__ src, int count, int nodeBase, uint32_t triBase, float4* __restrict__ dst )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= count) return;
	const float4* s = src + (size_t)i * 8;
	float4* d = dst + (size_t)(nodeBase + i) * 8;
	for (int k = 0; k < 6; k++) d[k] = s[k];
	const int4 r = *(const int4*)(s + 6);
	int ref[4] = { r.x, r.y, r.z, r.w };
	for (int c = 0; c < 4; c++) ref[c] = ref[c] >= 0 ? ref[c] + nodeBase : MAKE_LEAF( LEAF_FIRST( ref[c] ) + triBase, LEAF_COUNT( ref[c] ) );
	*(int4*)(d + 6) = make_int4( ref[0], ref[1], ref[2], ref[3] );
	d[7] = make_float4( 0, 0, 0, 0 );
}

/* TLAS (BVH2 at nodes2[base2 ...]) as BVH4 nodes of two children (slots 2, 3 empty) at
   nodes4[base4 ...]: interior references move from the BVH2 to the BVH4 index space, instance
   leaves stay; one node per thread, so per-frame TLAS updates cost one short launch */
__global__ __launch_bounds__( 256 ) void k_tlas_to_bvh4( const float4* __restrict__ nodes2, int base2, int count, int base4, float4* __restrict__ nodes4 )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= count) return;
	const float4* s = nodes2 + (size_t)(base2 + i) * 4;
	float4* d = nodes4 + (size_t)(base4 + i) * 8;
	const float nanv = __builtin_nanf( "" );
	/* BVH2 child pair (c0 lo.x hi.x lo.y hi.y | c1 ... | c0 lo.z hi.z c1 lo.z hi.z) -> the BVH4 planes */
	const float4 a = s[0], b = s[1], z = s[2];
	d[0] = make_float4( a.x, b.x, nanv, nanv ), d[1] = make_float4( a.y, b.y, nanv, nanv );
	d[2] = make_float4( a.z, b.z, nanv, nanv ), d[3] = make_float4( a.w, b.w, nanv, nanv );
	d[4] = make_float4( z.x, z.z, nanv, nanv ), d[5] = make_float4( z.y, z.w, nanv, nanv );
	const float4 r = s[3];
	int ref[2] = { __float_as_int( r.x ), __float_as_int( r.y ) };
	for (int c = 0; c < 2; c++) if (ref[c] >= 0) ref[c] = ref[c] - base2 + base4;
	*(int4*)(d + 6) = make_int4( ref[0], ref[1], MAKE_LEAF( 0, 1 ), MAKE_LEAF( 0, 1 ) );
	d[7] = make_float4( 0, 0, 0, 0 );
}

/* quantized BVH4 node (64 B, read by box4q in lh2_box4.inc):
     uint4 [0]  origin x, y, z (f32 bits: the smallest lo of the node's children), then the x grid step 2^e_x (f32 bits;
                plane = origin + q * 2^e)
     uint4 [1]  x lo bytes of children 0..3, x hi bytes, y lo bytes, y hi bytes
     uint4 [2]  z lo bytes, z hi bytes, the y and z grid steps 2^e_y, 2^e_z (f32 bits; round 6: exponent bytes before, which
                cost box4q a bit-field extract and an ldexp per axis, 4-cycle instructions, where a multiply is a 2-cycle one)
     uint4 [3]  the four child references (as the f32 node's)
   Child planes round outward (lo down, hi up, computed in double, so the quantized box holds the f32 one
   exactly); an empty slot (NaN planes) is the inverted box lo = 255, hi = 0 with the pop marker as its
   reference.  A box the traversal enters by mistake only costs work: it holds no hit the f32 tree's boxes
   do not hold (tests are exact per triangle).  Each exponent is at least the coordinate magnitude's - 28, so a plane's grid step is never
   below the rounding of the slab arithmetic, and at least -100 (the scaled reciprocal stays normal).  It is at most
   LH2_QEXP_MAX = 27: box4q scales the ray's reciprocal by 2^e, and an axis-parallel ray's reciprocal is clamped to
   +-1e30 (fast_inv), so 1e30 * 2^27 = 1.3e38 stays finite (a larger e makes it inf, and a zero byte plane times
   inf a NaN slab).  A node that would need more (extent > 255 * 2^27 = 3.4e10, or coordinates beyond 2^55) sets
   bit LH2_SCENE_ERR_QRANGE of the scene error flag, and the traversal kernels refuse the scene. */
__global__ __launch_bounds__( 256 ) void k_quantize4( const float4* __restrict__ nodes4, int first, int count, uint4* __restrict__ q, int* __restrict__ err )
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= count) return;
	const float4* s = nodes4 + (size_t)(first + i) * 8;
	float lo[3][4], hi[3][4];
	for (int a = 0; a < 3; a++)
	{
		const float4 l = s[2 * a], h = s[2 * a + 1];
		lo[a][0] = l.x, lo[a][1] = l.y, lo[a][2] = l.z, lo[a][3] = l.w;
		hi[a][0] = h.x, hi[a][1] = h.y, hi[a][2] = h.z, hi[a][3] = h.w;
	}
	bool valid[4];
	for (int c = 0; c < 4; c++)
	{
		valid[c] = true;
		for (int a = 0; a < 3; a++) valid[c] = valid[c] && isfinite( lo[a][c] ) && isfinite( hi[a][c] ) && lo[a][c] <= hi[a][c];
	}
	float origin[3];
	int e[3];
	uint32_t qlo[3] = { 0, 0, 0 }, qhi[3] = { 0, 0, 0 };
	for (int a = 0; a < 3; a++)
	{
		float o = 0, m = 0;
		bool any = false;
		for (int c = 0; c < 4; c++)
			if (valid[c]) o = any ? fminf( o, lo[a][c] ) : lo[a][c], m = any ? fmaxf( m, hi[a][c] ) : hi[a][c], any = true;
		origin[a] = o;
		const double ext = (double)m - (double)o;
		const double mag = fmax( fabs( (double)o ), fabs( (double)m ) );
		int ea = -100;
		if (ext > 0) ea = max( ea, (int)ceil( log2( ext / 255.0 ) ) );
		if (mag > 0) ea = max( ea, (int)floor( log2( mag ) ) - 28 );
		while (ext > 255.0 * ldexp( 1.0, ea ) && ea <= LH2_QEXP_MAX) ea++;   /* finite ext: ends at the cap at the latest */
		if (ea > LH2_QEXP_MAX) atomicOr( err, LH2_SCENE_ERR_QRANGE ), ea = LH2_QEXP_MAX;
		e[a] = ea;
		const double step = ldexp( 1.0, ea );
		for (int c = 0; c < 4; c++)
		{
			uint32_t l = 255, h = 0;
			if (valid[c])
			{
				const double dl = floor( ((double)lo[a][c] - (double)o) / step ), dh = ceil( ((double)hi[a][c] - (double)o) / step );
				l = (uint32_t)fmin( fmax( dl, 0.0 ), 255.0 ), h = (uint32_t)fmin( fmax( dh, 0.0 ), 255.0 );
				/* outward in exact arithmetic: origin + l * step <= lo, origin + h * step >= hi */
				while (l > 0 && (double)o + (double)l * step > (double)lo[a][c]) l--;
				while (h < 255 && (double)o + (double)h * step < (double)hi[a][c]) h++;
			}
			qlo[a] |= l << (8 * c), qhi[a] |= h << (8 * c);
		}
	}
	uint4* d = q + (size_t)(first + i) * 4;
	/* the grid steps 2^e as f32 (exact: -100 <= e <= LH2_QEXP_MAX): box4q scales the ray's reciprocal with one multiply */
	d[0] = make_uint4( __float_as_uint( origin[0] ), __float_as_uint( origin[1] ), __float_as_uint( origin[2] ), __float_as_uint( ldexpf( 1.0f, e[0] ) ) );
	d[1] = make_uint4( qlo[0], qhi[0], qlo[1], qhi[1] );
	d[2] = make_uint4( qlo[2], qhi[2], __float_as_uint( ldexpf( 1.0f, e[1] ) ), __float_as_uint( ldexpf( 1.0f, e[2] ) ) );
	/* an empty slot's reference is the traversal's pop marker (INT_MIN, LH2_POP in lh2_kernels.hip): if the
	   inverted box is ever entered (a small node far down the ray, where the exit pad exceeds its grid), the
	   ray just pops on (the f32 nodes keep 0 there, a real node, behind boxes of NaN that never hit) */
	int4 r = *(const int4*)(s + 6);
	if (!valid[0]) r.x = INT_MIN;
	if (!valid[1]) r.y = INT_MIN;
	if (!valid[2]) r.z = INT_MIN;
	if (!valid[3]) r.w = INT_MIN;
	d[3] = make_uint4( (uint32_t)r.x, (uint32_t)r.y, (uint32_t)r.z, (uint32_t)r.w );
}


inline int blocks( long n, int bs = 256 ) { return (int)std::max<long>( 1, (n + bs - 1) / bs ); }

}  // namespace

namespace lh2 {

/* the scratch is stream-ordered memory (hipMallocAsync / hipFreeAsync): a grown buffer's old block is freed on the stream
   of the last build that used it (lastStream: the TLAS builds run on the core's ahead stream, the BLAS builds on its core
   stream, and the callers order the two), so no device-wide synchronisation stalls the frames in flight */
template <class T> static void grow_buf( T*& p, size_t n, hipStream_t freeSt, hipStream_t st )
{
	if (p) CHK( hipFreeAsync( p, freeSt ) );
	CHK( hipMallocAsync( (void**)&p, std::max<size_t>( n, 1 ) * sizeof( T ), st ) );
}

GpuBvhBuilder::~GpuBvhBuilder()
{
	void* all[] = { boxes, prim, cl[0], cl[1], clNode[0], clNode[1], child, parent, P, I, cost, leafOrig, nn, keys[0], keys[1], vals[0], vals[1], flags, scan, dred, tmp };
	(void)hipDeviceSynchronize();
	for (void* p : all) if (p) (void)hipFreeAsync( p, nullptr );
	(void)hipStreamSynchronize( nullptr );
	if (hred) (void)hipHostFree( hred );
}

void GpuBvhBuilder::Reserve( int n, hipStream_t st )
{
	const hipStream_t freeSt = lastStream ? lastStream : st;
	retireStream = freeSt, lastStream = st;
	if (!dred)
	{
		CHK( hipMallocAsync( (void**)&dred, 16 * sizeof( uint32_t ), st ) );
		CHK( hipHostMalloc( (void**)&hred, 16 * sizeof( uint32_t ), hipHostMallocDefault ) );
	}
	if (n <= cap) return;
	/* the capacity grows by half again at least: a scene that keeps adding instances regrows O(log n) times */
	cap = std::max( n, std::max( 64, cap + cap / 2 ) );
	const size_t c = (size_t)cap, c2 = 2 * c;
	grow_buf( (Box8*&)boxes, c2, freeSt, st ); grow_buf( (Box8*&)prim, c, freeSt, st ); grow_buf( (Box8*&)cl[0], c, freeSt, st );
	grow_buf( (Box8*&)cl[1], c, freeSt, st ); grow_buf( clNode[0], c, freeSt, st ); grow_buf( clNode[1], c, freeSt, st );
	grow_buf( child, 2 * c2, freeSt, st ); grow_buf( parent, c2, freeSt, st ); grow_buf( P, c2, freeSt, st ); grow_buf( I, c2, freeSt, st );
	grow_buf( cost, c2, freeSt, st ); grow_buf( leafOrig, c, freeSt, st ); grow_buf( nn, c, freeSt, st ); grow_buf( keys[0], c, freeSt, st );
	grow_buf( keys[1], c, freeSt, st ); grow_buf( vals[0], c, freeSt, st ); grow_buf( vals[1], c, freeSt, st ); grow_buf( flags, c, freeSt, st );
	grow_buf( scan, c, freeSt, st );
}

/* the sort / scan temporaries, on the build's stream; a grown block's old one freed behind the previous build (Reserve) */
void* GpuBvhBuilder::Scratch( size_t bytes, hipStream_t st )
{
	if (bytes > tmpBytes)
	{
		if (tmp) CHK( hipFreeAsync( tmp, retireStream ) );
		tmpBytes = std::max<size_t>( bytes, std::max<size_t>( 1 << 20, tmpBytes + tmpBytes / 2 ) );
		CHK( hipMallocAsync( &tmp, tmpBytes, st ) );
	}
	return tmp;
}

/* Morton sort + PLOC rounds over the N primitive boxes in `prim` (bounds reduced into dred) */
void GpuBvhBuilder::Cluster( int N, int maxLeaf, float ct, int tlas, GpuBuildResult& res, hipStream_t st )
{
	Box8* pb = (Box8*)prim;
	k_morton<<<blocks( N ), 256, 0, st>>>( pb, N, dred, keys[0], vals[0] );
	size_t need = 0;
	CHK( hipcub::DeviceRadixSort::SortPairs( nullptr, need, keys[0], keys[1], vals[0], vals[1], N, 0, 63, st ) );
	size_t needScan = 0;
	CHK( hipcub::DeviceScan::ExclusiveSum( nullptr, needScan, flags, scan, N, st ) );
	void* t = Scratch( std::max( need, needScan ), st );
	CHK( hipcub::DeviceRadixSort::SortPairs( t, need, keys[0], keys[1], vals[0], vals[1], N, 0, 63, st ) );
	k_init_leaves<<<blocks( N ), 256, 0, st>>>( vals[1], pb, N, (Box8*)boxes, P, I, cost, parent, leafOrig, clNode[0], (Box8*)cl[0] );
	const int r = std::min( 32, std::max( 1, radius ) );
	int n = N, made = 0, cur = 0, rounds = 0;
	while (n > 1)
	{
		k_nn<<<blocks( n ), 256, 0, st>>>( (const Box8*)cl[cur], n, r, nn );
		k_flags<<<blocks( n ), 256, 0, st>>>( nn, n, flags );
		size_t sb = tmpBytes;
		CHK( hipcub::DeviceScan::ExclusiveSum( tmp, sb, flags, scan, n, st ) );
		k_merge<<<blocks( n ), 256, 0, st>>>( clNode[cur], (const Box8*)cl[cur], nn, flags, scan, n, N + made, maxLeaf, ct,
			clNode[1 - cur], (Box8*)cl[1 - cur], (Box8*)boxes, child, parent, P, I, cost, dred );
		CHK( hipMemcpyAsync( hred + 12, dred + 12, 2 * sizeof( uint32_t ), hipMemcpyDeviceToHost, st ) );
		CHK( hipStreamSynchronize( st ) );
		const int nn2 = (int)hred[12];
		if (nn2 >= n || hred[13] == 0) FatalError( "GPU BVH build made no progress (%d clusters)", n );
		n = nn2, made += (int)hred[13], cur = 1 - cur, rounds++;
	}
	res.rounds = rounds;
	(void)tlas;
}

void GpuBvhBuilder::BuildBlas( const float4* coreTris, int N, int maxLeaf, float ct, float4** nodesOut, float4** trisOut, GpuBuildResult& res, hipStream_t st )
{
	if (N < 2) FatalError( "GPU BLAS build needs >= 2 triangles" );
	maxLeaf = std::min( 16, std::max( 1, maxLeaf ) );
	Reserve( N, st );
	k_reset_red<<<1, 64, 0, st>>>( dred );
	k_tri_bounds<<<std::min( blocks( N ), 2048 ), 256, 0, st>>>( coreTris, N, (Box8*)prim, dred );
	Cluster( N, maxLeaf, ct, 0, res, st );
	const int root = 2 * N - 2;
	CHK( hipMemcpyAsync( hred + 15, I + root, sizeof( uint32_t ), hipMemcpyDeviceToHost, st ) );
	CHK( hipMemcpyAsync( hred, dred, 12 * sizeof( uint32_t ), hipMemcpyDeviceToHost, st ) );
	CHK( hipStreamSynchronize( st ) );
	res.nodeCount = (int)hred[15];
	for (int k = 0; k < 3; k++) res.lo[k] = o2f( hred[6 + k] ), res.hi[k] = o2f( hred[9 + k] );
	CHK( hipMalloc( (void**)nodesOut, (size_t)res.nodeCount * 4 * sizeof( float4 ) ) );
	CHK( hipMalloc( (void**)trisOut, (size_t)N * 3 * sizeof( float4 ) ) );
	k_emit<<<blocks( 2L * N - 1 ), 256, 0, st>>>( N, 0, 0, 0, (const Box8*)boxes, child, parent, P, I, leafOrig, coreTris, *nodesOut, *trisOut, dred );
	CHK( hipMemcpyAsync( hred + 14, dred + 14, sizeof( uint32_t ), hipMemcpyDeviceToHost, st ) );
	CHK( hipStreamSynchronize( st ) );
	res.maxDepth = (int)hred[14];
}

void GpuBvhBuilder::BuildTlas( const GpuTlasArgs& a, hipStream_t st )
{
	const int N = a.count;
	if (N < 2) FatalError( "GPU TLAS build needs >= 2 instances" );
	Reserve( N, st );
	if (N <= LH2_TLAS_WG_MAX)
	{
		TlasScratch s;
		s.prim = (Box8*)prim, s.boxes = (Box8*)boxes, s.cl0 = (Box8*)cl[0], s.cl1 = (Box8*)cl[1], s.clNode0 = clNode[0], s.clNode1 = clNode[1];
		s.child = child, s.parent = parent, s.P = P, s.I = I, s.cost = cost, s.leafOrig = leafOrig, s.nn = nn;
		k_tlas_build_wg<<<1, 1024, 0, st>>>( a, s, std::min( 32, std::max( 1, radius ) ) );
		return;
	}
	k_reset_red<<<1, 64, 0, st>>>( dred );
	k_inst_bounds<<<std::min( blocks( N ), 2048 ), 256, 0, st>>>( a.T, a.instMesh, a.meshBounds, N, (Box8*)prim, dred );
	GpuBuildResult res;
	Cluster( N, 1, 1.0f, 1, res, st );
	k_emit<<<blocks( 2L * N - 1 ), 256, 0, st>>>( N, 1, a.nodeBase, 0, (const Box8*)boxes, child, parent, P, I, leafOrig, nullptr, a.nodes, nullptr, dred );
	k_tlas_check<<<1, 1, 0, st>>>( dred, a.maxBlasDepth, a.tlasFactor, a.sceneError, a.tlasDepth );
}

void GpuBvhBuilder::Relocate( const float4* src, int nodeCount, int nodeBase, uint32_t triBase, float4* dst, hipStream_t st )
{
	if (nodeCount <= 0) return;
	k_relocate<<<blocks( nodeCount ), 256, 0, st>>>( src, nodeCount, nodeBase, triBase, dst );
}
void GpuBvhBuilder::Relocate4( const float4* src, int nodeCount, int nodeBase, uint32_t triBase, float4* dst, hipStream_t st )
{
	if (nodeCount <= 0) return;
	k_relocate4<<<blocks( nodeCount ), 256, 0, st>>>( src, nodeCount, nodeBase, triBase, dst );
}
void GpuBvhBuilder::Quantize4( const float4* nodes4, int first, int count, uint4* q, int* sceneError, hipStream_t st )
{
	if (count <= 0) return;
	k_quantize4<<<blocks( count ), 256, 0, st>>>( nodes4, first, count, q, sceneError );
	CHK( hipGetLastError() );
}

void GpuBvhBuilder::TlasToBvh4( const float4* nodes2, int base2, int count, int base4, float4* nodes4, hipStream_t st )
{
	if (count <= 0) return;
	k_tlas_to_bvh4<<<blocks( count ), 256, 0, st>>>( nodes2, base2, count, base4, nodes4 );
}

}  // namespace lh2
