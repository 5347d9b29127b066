/* bvh_check.cpp - host-side invariants of the core's BLAS builder (bvh_build.cpp), run by tests/test_bvh_host.py on the
   CPU: for a seeded triangle soup and a seeded grid of small triangles, built with and without spatial splits (SBVH),
     1. every triangle is referenced by at least one leaf (out.perm), and every leaf slot names a real triangle;
     2. coverage: sample points on every triangle (its vertices, edge midpoints and seeded interior points) are each
        reachable from the root through child boxes that contain them (closed boxes, exact compares) down to a leaf
        that references that triangle: a ray that hits the triangle there enters every box on the way, so the
        traversal reaches the triangle (the spatial splits clip references at planes: the clipped boxes must still
        cover the triangle, bvh_build.cpp split_ref);
     3. the reported depth bounds the real depth.
   Prints one line per build ("ok" or the first failures) and exits nonzero on any failure.
   Build: g++ -O2 -std=c++17 -pthread tools/bvh_check.cpp lighthouse2_amd/csrc/bvh_build.cpp -o bvh_check */
#include "../lighthouse2_amd/csrc/bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace lh2;

namespace {

uint32_t xs( uint32_t& s ) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }
float uf( uint32_t& s ) { return (float)(xs( s ) >> 8) * (1.0f / 16777216.0f); }

/* kind 0: config 2's triangle soup (many overlapping triangles: the spatial splits' case); kind 1: small triangles on a grid */
std::vector<float> make_tris( int n, int kind, uint32_t seed )
{
	std::vector<float> v( (size_t)n * 9 );
	uint32_t s = seed;
	const int g = 1 + (int)std::sqrt( (double)n );
	for (int i = 0; i < n; i++)
	{
		float* t = &v[(size_t)i * 9];
		if (kind == 0)
		{
			/* v0 uniform in a cube, edges 0.5 (scene.random_triangles), the cube sized for config 2's density at n = 100k */
			const float side = 10.0f * (float)std::cbrt( n / 100000.0 );
			for (int k = 0; k < 3; k++) t[k] = (uf( s ) - 0.5f) * side;
			for (int k = 3; k < 9; k++) t[k] = t[k % 3] + (uf( s ) - 0.5f) * 0.5f;
		}
		else
		{
			const float x = (float)(i % g), z = (float)(i / g);
			const float p[9] = { x, 0, z, x + 1, 0.1f * uf( s ), z, x, 0.1f * uf( s ), z + 1 };
			memcpy( t, p, sizeof( p ) );
		}
	}
	return v;
}

struct Checker
{
	const BvhOutput& b;
	explicit Checker( const BvhOutput& bv ) : b( bv ) {}
	static bool in( const float p[3], float lx, float hx, float ly, float hy, float lz, float hz )
	{
		return p[0] >= lx && p[0] <= hx && p[1] >= ly && p[1] <= hy && p[2] >= lz && p[2] <= hz;
	}
	bool leaf_has( int ref, uint32_t prim ) const
	{
		const uint32_t first = LEAF_FIRST_( ref ), count = LEAF_COUNT_( ref );
		for (uint32_t i = 0; i < count; i++) if (b.perm[first + i] == prim) return true;
		return false;
	}
	static uint32_t LEAF_FIRST_( int ref ) { return (uint32_t)(~ref) >> 4; }
	static uint32_t LEAF_COUNT_( int ref ) { return ((uint32_t)(~ref) & 15u) + 1; }
	/* is prim reachable at point p from node k (its two children's boxes hold in the node) */
	bool reach( int k, const float p[3], uint32_t prim, int depth, int& maxDepth ) const
	{
		maxDepth = std::max( maxDepth, depth );
		const float* n = &b.nodes[(size_t)k * 16];
		int refs[2];
		memcpy( refs, n + 12, 8 );
		const bool inA = in( p, n[0], n[1], n[2], n[3], n[8], n[9] ), inB = in( p, n[4], n[5], n[6], n[7], n[10], n[11] );
		for (int c = 0; c < 2; c++)
		{
			if (!(c ? inB : inA)) continue;
			if (refs[c] >= 0) { if (reach( refs[c], p, prim, depth + 1, maxDepth )) return true; }
			else if (leaf_has( refs[c], prim )) return true;
		}
		return false;
	}
};

int check( const char* name, const std::vector<float>& tv, float alpha, int minRefs )
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
	BuildBvh2( prims, 1, 4, b, 1.0f, 0, alpha > 0 ? tv.data() : nullptr, alpha, 1.0f, minRefs );
	int fails = 0;
	std::vector<int> seen( n, 0 );
	for (uint32_t p : b.perm)
	{
		if (p >= (uint32_t)n) { if (fails++ < 5) std::printf( "  %s: leaf slot names triangle %u of %d\n", name, p, n ); continue; }
		seen[p] = 1;
	}
	for (int i = 0; i < n; i++) if (!seen[i] && fails++ < 5) std::printf( "  %s: triangle %d in no leaf\n", name, i );
	Checker ck( b );
	uint32_t s = 0x9e3779b9u;
	int maxDepth = 0;
	long points = 0;
	for (int i = 0; i < n; i++)
	{
		const float* t = &tv[(size_t)i * 9];
		float bary[9][2] = { { 0, 0 }, { 1, 0 }, { 0, 1 }, { 0.5f, 0 }, { 0, 0.5f }, { 0.5f, 0.5f }, { 0, 0 }, { 0, 0 }, { 0, 0 } };
		for (int j = 6; j < 9; j++) { float u = uf( s ), v = uf( s ); if (u + v > 1) u = 1 - u, v = 1 - v; bary[j][0] = u, bary[j][1] = v; }
		for (int j = 0; j < 9; j++)
		{
			const float u = bary[j][0], v = bary[j][1];
			float p[3];
			for (int k = 0; k < 3; k++) p[k] = j == 0 ? t[k] : j == 1 ? t[3 + k] : j == 2 ? t[6 + k] : t[k] + u * (t[3 + k] - t[k]) + v * (t[6 + k] - t[k]);
			points++;
			if (!ck.reach( 0, p, (uint32_t)i, 1, maxDepth ) && fails++ < 5)
				std::printf( "  %s: triangle %d point %d (%g %g %g) not reachable\n", name, i, j, p[0], p[1], p[2] );
		}
	}
	if (maxDepth > b.maxDepth && fails++ < 5) std::printf( "  %s: depth %d beyond the reported %d\n", name, maxDepth, b.maxDepth );
	std::printf( "%s: tris %d refs %zu nodes %zu depth %d points %ld %s\n", name, n, b.perm.size(), b.nodes.size() / 16, b.maxDepth, points,
		fails ? "FAIL" : "ok" );
	return fails;
}

}  // namespace

int main( int argc, char** argv )
{
	const int n = argc > 1 ? atoi( argv[1] ) : 20000;
	int fails = 0;
	for (int kind = 0; kind < 2; kind++)
	{
		const std::vector<float> tv = make_tris( n, kind, 0x12345678u + kind );
		char name[64];
		std::snprintf( name, sizeof( name ), "%s sah", kind ? "grid" : "soup" );
		fails += check( name, tv, 0.0f, 0 );
		std::snprintf( name, sizeof( name ), "%s sbvh 1e-3", kind ? "grid" : "soup" );
		fails += check( name, tv, 1e-3f, 0 );
		std::snprintf( name, sizeof( name ), "%s sbvh 1e-5", kind ? "grid" : "soup" );
		fails += check( name, tv, 1e-5f, 0 );
		std::snprintf( name, sizeof( name ), "%s sbvh 1e-3 min64", kind ? "grid" : "soup" );
		fails += check( name, tv, 1e-3f, 64 );
	}
	return fails ? 1 : 0;
}
