/* w8_check.cpp - host checks of the W8 builder (bvh_build.cpp BuildW8, lh2_w8.h), no GPU (tests/test_bvh_host.py):
   for a config-2-density triangle soup (SBVH at the default threshold) and a grid of small triangles,
   1. every triangle sits in exactly the leaf slots of the BVH2's leaves, and sample points on it (vertices, edge midpoints,
      seeded interior points) reach a triangle record holding it through dequantized child boxes that contain them;
   2. closest hits of seeded random rays through the W8, traversed as the GPU loop does (node groups on a stack, slots in
      the key order slot ^ octant, the interior mask of the ray's octant, leaf groups, exact slab tests against the
      dequantized planes), equal the brute-force closest hits (t, then triangle) of the same Moller-Trumbore test;
   3. the reported W8 depth bounds the real one.
   Prints one line per build ending in "ok" or "FAIL". */
#include "../lighthouse2_amd/csrc/bvh_build.h"
#include "../lighthouse2_amd/csrc/lh2_w8.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace lh2;

namespace {

float uf( uint32_t& s ) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return (float)(s >> 8) * (1.0f / 16777216.0f); }

struct W8View
{
	const std::vector<uint32_t>& r;
	explicit W8View( const std::vector<uint32_t>& rec ) : r( rec ) {}
	const uint32_t* rec( size_t i ) const { return &r[i * LH2_W8_WORDS]; }
	/* the dequantized box of slot s of node record n (double, as k_quantize4 rounds: origin + q * 2^e) */
	void box( const uint32_t* n, int s, double lo[3], double hi[3] ) const
	{
		for (int a = 0; a < 3; a++)
		{
			float o;
			memcpy( &o, &n[a], 4 );
			const int e = (int)(int8_t)((n[3] >> (8 * a)) & 255u);
			const uint32_t lw = n[4 + 4 * a + (s >> 2)], hw = n[6 + 4 * a + (s >> 2)];
			lo[a] = (double)o + (double)((lw >> (8 * (s & 3))) & 255u) * std::ldexp( 1.0, e );
			hi[a] = (double)o + (double)((hw >> (8 * (s & 3))) & 255u) * std::ldexp( 1.0, e );
		}
	}
	uint32_t imask( const uint32_t* n ) const { return n[16] & 255u; }   /* octant 0: key order = slot order */
};

/* Bart's common.h:19-50 Moller-Trumbore (open interval, as the oracle's intersect_tri) on the 48-B record */
bool mt( const float* t, const float o[3], const float d[3], float& tt )
{
	const float* v0 = t; const float* e1 = t + 4; const float* e2 = t + 8;
	const float h[3] = { d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0] };
	const float det = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
	if (det == 0.0f) return false;
	const float f = 1.0f / det;
	const float s[3] = { o[0] - v0[0], o[1] - v0[1], o[2] - v0[2] };
	const float u = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
	if (u < 0.0f || u > 1.0f) return false;
	const float q[3] = { s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0] };
	const float v = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
	if (v < 0.0f || u + v > 1.0f) return false;
	tt = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
	return tt > 0.0f;
}

bool slab( const double lo[3], const double hi[3], const float o[3], const float d[3], double tmax )
{
	double t0 = 0, t1 = tmax;
	for (int a = 0; a < 3; a++)
	{
		if (d[a] == 0.0f) { if (o[a] < lo[a] || o[a] > hi[a]) return false; continue; }
		double ta = (lo[a] - o[a]) / d[a], tb = (hi[a] - o[a]) / d[a];
		if (ta > tb) std::swap( ta, tb );
		t0 = std::max( t0, ta ), t1 = std::min( t1, tb * (1 + 1e-9) + 1e-12 );
	}
	return t0 <= t1;
}

int check( const char* name, const std::vector<float>& tv, float alpha )
{
	const int n = (int)(tv.size() / 9);
	std::vector<Aabb> prims( n );
	for (int i = 0; i < n; i++)
		for (int k = 0; k < 3; k++)
		{
			const float* t = &tv[(size_t)i * 9];
			prims[i].lo[k] = std::min( std::min( t[k], t[3 + k] ), t[6 + k] );
			prims[i].hi[k] = std::max( std::max( t[k], t[3 + k] ), t[6 + k] );
		}
	BvhOutput b;
	BuildBvh2( prims, 1, 4, b, 1.0f, 0, alpha > 0 ? tv.data() : nullptr, alpha, 1.0f, 64 );
	std::vector<float> t48( b.perm.size() * 12, 0.0f );
	for (size_t j = 0; j < b.perm.size(); j++)
	{
		const float* v = &tv[(size_t)b.perm[j] * 9];
		float* o = &t48[j * 12];
		o[0] = v[0], o[1] = v[1], o[2] = v[2]; memcpy( &o[3], &b.perm[j], 4 );
		for (int k = 0; k < 3; k++) o[4 + k] = v[3 + k] - v[k], o[8 + k] = v[6 + k] - v[k];
	}
	std::vector<uint32_t> rec;
	int blocks = 0, depth = 0, qerr = 0, fails = 0;
	if (!BuildW8( b.nodes.data(), b.nodes.size() / 16, t48.data(), b.perm.size(), 0.4f, 0.5f, rec, blocks, depth, qerr ))
	{
		std::printf( "%s: BuildW8 refused FAIL\n", name );
		return 1;
	}
	if (qerr && fails++ < 5) std::printf( "  %s: quantizer range error\n", name );
	W8View w( rec );
	/* 1. every leaf slot's triangle is a BVH2 leaf triangle, each triangle appears as often as in the BVH2's leaves; and
	   reachability of sample points */
	std::vector<int> inW8( n, 0 ), inBvh( n, 0 );
	for (uint32_t p : b.perm) inBvh[p]++;
	int maxDepth = 0;
	std::vector<std::pair<size_t, int>> stack{ { 0, 1 } };
	long leaves = 0;
	while (!stack.empty())
	{
		const auto [ri, d] = stack.back();
		stack.pop_back();
		maxDepth = std::max( maxDepth, d );
		const uint32_t* nr = w.rec( ri );
		const uint32_t im = w.imask( nr );
		for (int s = 0; s < 8; s++)
		{
			double lo[3], hi[3];
			w.box( nr, s, lo, hi );
			if (lo[0] > hi[0]) continue;   /* an empty slot: inverted box */
			const size_t ci = (size_t)nr[18] * 8 + (size_t)s;
			if (ci * LH2_W8_WORDS >= rec.size()) { if (fails++ < 5) std::printf( "  %s: child record %zu beyond the array\n", name, ci ); continue; }
			if ((im >> s) & 1u) stack.push_back( { ci, d + 1 } );
			else
			{
				uint32_t tri;
				memcpy( &tri, &w.rec( ci )[3], 4 );
				if (tri >= (uint32_t)n) { if (fails++ < 5) std::printf( "  %s: leaf names triangle %u\n", name, tri ); continue; }
				inW8[tri]++, leaves++;
			}
		}
	}
	for (int i = 0; i < n; i++) if (inW8[i] != inBvh[i] && fails++ < 5) std::printf( "  %s: triangle %d in %d W8 leaves, %d BVH2 leaves\n", name, i, inW8[i], inBvh[i] );
	if (maxDepth > depth + 1 && fails++ < 5) std::printf( "  %s: depth %d beyond the reported %d\n", name, maxDepth, depth );
	/* 2. rays: the GPU loop's order and groups against brute force */
	uint32_t s = 0x2545f491u;
	float lo[3] = { 1e30f, 1e30f, 1e30f }, hi[3] = { -1e30f, -1e30f, -1e30f };
	for (size_t i = 0; i < tv.size(); i++) lo[i % 3] = std::min( lo[i % 3], tv[i] ), hi[i % 3] = std::max( hi[i % 3], tv[i] );
	const int rays = 3000;
	long steps = 0;
	for (int r = 0; r < rays; r++)
	{
		float o[3], tg[3], d[3];
		for (int a = 0; a < 3; a++) o[a] = lo[a] + (hi[a] - lo[a]) * (1.5f * uf( s ) - 0.25f), tg[a] = lo[a] + (hi[a] - lo[a]) * uf( s );
		float len = 0;
		for (int a = 0; a < 3; a++) d[a] = tg[a] - o[a], len += d[a] * d[a];
		len = std::sqrt( len );
		for (int a = 0; a < 3; a++) d[a] /= len;
		if (r % 7 == 0) d[r % 3] = 0.0f;   /* axis-parallel components */
		/* brute force */
		float bt = 1e30f; uint32_t btri = 0xffffffffu;
		for (size_t j = 0; j < b.perm.size(); j++)
		{
			float t;
			if (mt( &t48[j * 12], o, d, t ) && (t < bt || (t == bt && b.perm[j] < btri))) bt = t, btri = b.perm[j];
		}
		/* the W8 walk */
		const uint32_t m = (d[0] > 0 ? 1u : 0u) | (d[1] > 0 ? 2u : 0u) | (d[2] > 0 ? 4u : 0u);
		float wt = 1e30f; uint32_t wtri = 0xffffffffu;
		std::vector<uint32_t> st;
		long node = 0;   /* the record to step, -1: pop */
		while (true)
		{
			if (node >= 0)
			{
				steps++;
				const uint32_t* nr = w.rec( (size_t)node );
				uint32_t hm = 0;
				for (int k = 0; k < 8; k++)
				{
					double blo[3], bhi[3];
					w.box( nr, k, blo, bhi );
					if (blo[0] <= bhi[0] && slab( blo, bhi, o, d, wt )) hm |= 1u << k;
				}
				uint32_t hk = 0;
				for (int k = 0; k < 8; k++) if ((hm >> k) & 1u) hk |= 1u << (k ^ m);
				const uint32_t ik = ((m & 4) ? nr[17] : nr[16]) >> (8 * (m & 3)) & 255u;
				uint32_t nodeK = hk & ik, leafK = hk & ~ik & 255u;
				const uint32_t blk = nr[18];
				node = -1;
				/* the leaves at once (the GPU parks them; the hits do not depend on when they are tested) */
				for (; leafK; leafK &= leafK - 1)
				{
					const uint32_t* tr = w.rec( (size_t)blk * 8 + ((uint32_t)__builtin_ctz( leafK ) ^ m) );
					float t;
					uint32_t tri;
					memcpy( &tri, &tr[3], 4 );
					if (mt( (const float*)tr, o, d, t ) && (t < wt || (t == wt && tri < wtri))) wt = t, wtri = tri;
				}
				if (nodeK)
				{
					node = (long)blk * 8 + ((uint32_t)__builtin_ctz( nodeK ) ^ m);
					nodeK &= nodeK - 1;
					if (nodeK) st.push_back( (blk << 9) | nodeK );
				}
			}
			else
			{
				if (st.empty()) break;
				uint32_t& e = st.back();
				node = (long)(e >> 9) * 8 + ((uint32_t)__builtin_ctz( e ) ^ m);
				e &= e - 1;
				if (!(e & 255u)) st.pop_back();
			}
		}
		if ((wtri != btri || (btri != 0xffffffffu && wt != bt)) && fails++ < 5)
			std::printf( "  %s: ray %d: W8 hit %u t %.9g, brute force %u t %.9g\n", name, r, wtri, wt, btri, bt );
	}
	std::printf( "%s: tris %d refs %zu blocks %d depth %d leaves %ld node steps/ray %.2f %s\n", name, n, b.perm.size(), blocks, depth, leaves,
		(double)steps / rays, fails ? "FAIL" : "ok" );
	return fails;
}

}  // namespace

int main( int argc, char** argv )
{
	const int n = argc > 1 ? atoi( argv[1] ) : 20000;
	int fails = 0;
	/* a triangle soup at config 2's density (xorshift, 10^3 box, edges 0.5 scaled to the count) */
	{
		std::vector<float> tv( (size_t)n * 9 );
		uint32_t s = 0x12345678u;
		const float edge = 0.5f * std::cbrt( 100000.0f / (float)n );
		for (int i = 0; i < n; i++)
		{
			float v0[3];
			for (int k = 0; k < 3; k++) v0[k] = uf( s ) * 10.0f - 5.0f;
			for (int k = 0; k < 3; k++) tv[(size_t)i * 9 + k] = v0[k];
			for (int k = 0; k < 3; k++) tv[(size_t)i * 9 + 3 + k] = v0[k] + (uf( s ) - 0.5f) * edge;
			for (int k = 0; k < 3; k++) tv[(size_t)i * 9 + 6 + k] = v0[k] + (uf( s ) - 0.5f) * edge;
		}
		fails += check( "soup sah", tv, 0.0f );
		fails += check( "soup sbvh 1e-3", tv, 1e-3f );
	}
	/* a grid of small triangles (many equal boxes along two axes) */
	{
		const int g = (int)std::sqrt( (double)n / 2 );
		std::vector<float> tv;
		for (int i = 0; i < g; i++)
			for (int j = 0; j < g; j++)
			{
				const float x = (float)i * 0.1f, z = (float)j * 0.1f;
				const float a[9] = { x, 0, z, x + 0.1f, 0, z, x, 0, z + 0.1f }, c[9] = { x + 0.1f, 0, z, x + 0.1f, 0.01f, z + 0.1f, x, 0, z + 0.1f };
				tv.insert( tv.end(), a, a + 9 ), tv.insert( tv.end(), c, c + 9 );
			}
		fails += check( "grid sah", tv, 0.0f );
	}
	return fails ? 1 : 0;
}
