/* wave_sim.cpp - host-side model of the BVH4 loop's wave behaviour (tools only, no GPU): one persistent wave of 64
   lanes runs the loop of lh2_trace4d.inc (refill once `refill` lanes are idle, the one-entry leaf slot with batches
   of `leafBatch` parked leaves, the pop, the queue-dry policies) over bounce stand-in rays of the config-2 soup, on
   the core's tree (SBVH 1e-3 + the DP BVH4 collapse), with exact f32 slab tests.  It counts what the GPU's
   LH2_TRACE_STATS counts (iterations, active lanes, node steps and their lanes, leaf passes and their lanes, refills)
   and prices an iteration with the ISA's per-block VALU counts of k_trace_closest4d<true> (loop control 25, node
   step + pushes 117, leaf pass 74 per triangle, pop 20, a second pop 20, refill 87): a model to rank loop policies
   before building them, not a timing.
     variants: base, pop-through (a popped BLAS leaf parked at once when the slot is free, then pop again),
     slot2 (a two-entry leaf slot).
   Build: g++ -O2 -std=c++17 -pthread tools/wave_sim.cpp lighthouse2_amd/csrc/bvh_build.cpp -o /tmp/wave_sim
   Run:   /tmp/wave_sim tris.bin [rays] [refill] [leafBatch] */
#include "../lighthouse2_amd/csrc/bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using namespace lh2;

namespace {

struct V3 { float x, y, z; };
V3 sub( V3 a, V3 b ) { return { a.x - b.x, a.y - b.y, a.z - b.z }; }
V3 cross( V3 a, V3 b ) { return { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x }; }
float dot( V3 a, V3 b ) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 norm( V3 a ) { const float l = std::sqrt( dot( a, a ) ); return { a.x / l, a.y / l, a.z / l }; }

constexpr int POP = INT32_MIN, FIN = INT32_MIN + 1;
bool is_leaf( int n ) { return n < 0 && n != POP && n != FIN; }

struct Ray { V3 o, d, id; };

struct Model
{
	std::vector<float> tv, n4;
	std::vector<uint32_t> perm;
	void tri( uint32_t t, const Ray& r, float& tb ) const
	{
		const float* v = &tv[(size_t)t * 9];
		const V3 v0 = { v[0], v[1], v[2] }, e1 = sub( { v[3], v[4], v[5] }, v0 ), e2 = sub( { v[6], v[7], v[8] }, v0 );
		const V3 p = cross( r.d, e2 );
		const float det = dot( e1, p );
		if (std::fabs( det ) < 1e-12f) return;
		const float inv = 1.0f / det;
		const V3 s = sub( r.o, v0 );
		const float u = dot( s, p ) * inv;
		if (u < 0 || u > 1) return;
		const V3 q = cross( s, e1 );
		const float w = dot( r.d, q ) * inv;
		if (w < 0 || u + w > 1) return;
		const float tt = dot( e2, q ) * inv;
		if (tt > 1e-4f && tt < tb) tb = tt;
	}
	/* the node step: entered children nearest first */
	int step( int node, const Ray& r, float tb, int* out ) const
	{
		const float* q = &n4[(size_t)node * 32];
		const int* refs = (const int*)(q + 24);
		float tn[4]; int nh = 0;
		for (int c = 0; c < 4; c++)
		{
			const float lx = q[c], hx = q[4 + c], ly = q[8 + c], hy = q[12 + c], lz = q[16 + c], hz = q[20 + c];
			if (!(lx == lx)) continue;
			const float ax = (lx - r.o.x) * r.id.x, bx = (hx - r.o.x) * r.id.x, ay = (ly - r.o.y) * r.id.y, by = (hy - r.o.y) * r.id.y;
			const float az = (lz - r.o.z) * r.id.z, bz = (hz - r.o.z) * r.id.z;
			const float n = std::fmax( std::fmax( std::fmin( ax, bx ), std::fmin( ay, by ) ), std::fmax( std::fmin( az, bz ), 0.0f ) );
			const float f = std::fmin( std::fmin( std::fmax( ax, bx ), std::fmax( ay, by ) ), std::fmax( az, bz ) );
			if (n <= f * 1.00001f && n <= tb) { tn[nh] = n, out[nh] = refs[c]; nh++; }
		}
		for (int i = 1; i < nh; i++)
			for (int k = i; k > 0 && tn[k] < tn[k - 1]; k--) std::swap( tn[k], tn[k - 1] ), std::swap( out[k], out[k - 1] );
		return nh;
	}
};

struct Lane
{
	bool act = false;
	int node = POP, sp = 0, leaf[2] = { 0, 0 };
	int stack[256];
	float tb = 1e30f;
	Ray r;
	int nleaf() const { return (leaf[0] != 0) + (leaf[1] != 0); }
};

struct Counts { double iters = 0, active = 0, nodeIters = 0, nodeLanes = 0, leafPasses = 0, leafLanes = 0, leafTris = 0, refills = 0, pops2 = 0, valu = 0, valuLanes = 0; };

/* variant: 0 base, 1 pop-through, 2 two-entry leaf slot */
Counts simulate( const Model& m, const std::vector<Ray>& rays, int variant, int refill, int leafBatch )
{
	Counts c;
	Lane L[64];
	size_t next = 0;
	bool exhausted = false;
	const int slots = variant == 2 ? 2 : 1;
	auto valu = [&]( double n, int lanes ) { c.valu += n; c.valuLanes += n * lanes; };
	while (true)
	{
		int idle = 0;
		for (auto& l : L) idle += !l.act;
		if (!exhausted && idle >= refill)
		{
			int got = 0;
			for (auto& l : L)
				if (!l.act)
				{
					if (next >= rays.size()) { exhausted = true; break; }
					l = Lane();
					l.act = true, l.r = rays[next++], l.node = 0, l.sp = 0, l.tb = 1e30f;
					got++;
				}
			if (got) { c.refills++; valu( 87, got ); }
		}
		int act = 0;
		for (auto& l : L) act += l.act;
		if (exhausted && act == 0) break;
		c.iters++, c.active += act;
		valu( 25, act );
		/* leaf phase */
		int leafLanes = 0, blockedOrDone = 0, walking = 0;
		for (auto& l : L)
			if (l.act)
			{
				walking++;
				const bool has = l.nleaf() > 0;
				leafLanes += has;
				const bool full = l.nleaf() == slots;
				const bool blocked = has && ((is_leaf( l.node ) && full) || (l.node == POP && l.sp == 0));
				blockedOrDone += blocked;
			}
		bool doLeaf = leafLanes >= (exhausted ? 1 : leafBatch);
		if (!doLeaf && leafLanes) doLeaf = blockedOrDone == walking;
		if (doLeaf && leafLanes)
		{
			int maxT = 0;
			for (auto& l : L)
				if (l.act && l.nleaf())
				{
					int nt = 0;
					for (int s = 0; s < 2; s++)
						if (l.leaf[s])
						{
							const uint32_t first = (uint32_t)(~l.leaf[s]) >> 4;
							const int cnt = (int)((uint32_t)(~l.leaf[s]) & 15u) + 1;
							for (int k = 0; k < cnt; k++) m.tri( m.perm[first + k], l.r, l.tb ), nt++;
							l.leaf[s] = 0;
						}
					maxT = std::max( maxT, nt );
					c.leafTris += nt;
				}
			c.leafPasses++, c.leafLanes += leafLanes;
			valu( 74.0 * maxT, leafLanes );
		}
		/* node step */
		int nodeLanes = 0;
		for (auto& l : L) nodeLanes += l.act && l.node >= 0;
		if (nodeLanes)
		{
			c.nodeIters++, c.nodeLanes += nodeLanes;
			valu( 117, nodeLanes );
			for (auto& l : L)
				if (l.act && l.node >= 0)
				{
					int ch[4];
					const int nh = m.step( l.node, l.r, l.tb, ch );
					l.node = nh ? ch[0] : POP;
					for (int i = nh - 1; i >= 1; i--) l.stack[l.sp++] = ch[i];
					if (is_leaf( l.node ) && l.nleaf() < slots) { l.leaf[l.leaf[0] ? 1 : 0] = l.node; l.node = POP; }
				}
		}
		/* a BLAS leaf reached by a pop: park it (a full slot: wait) */
		for (auto& l : L)
			if (l.act && is_leaf( l.node ) && l.nleaf() < slots) { l.leaf[l.leaf[0] ? 1 : 0] = l.node; l.node = POP; }
		/* pop */
		int popLanes = 0, pop2 = 0;
		for (auto& l : L)
			if (l.act && l.node == POP && !(l.nleaf() && l.sp == 0))
			{
				popLanes++;
				if (l.sp == 0) l.node = FIN;
				else l.node = l.stack[--l.sp];
				if (variant == 1 && is_leaf( l.node ) && l.nleaf() < slots)
				{
					pop2++;
					l.leaf[0] = l.node;
					l.node = l.sp == 0 ? POP : l.stack[--l.sp];
				}
			}
		if (popLanes) valu( 20, popLanes );
		if (pop2) { valu( 20, pop2 ); c.pops2++; }
		for (auto& l : L)
			if (l.act && l.node == FIN) l.act = false;
	}
	return c;
}

}  // namespace

int main( int argc, char** argv )
{
	if (argc < 2) { std::fprintf( stderr, "usage: wave_sim tris.bin [rays] [refill] [leafBatch]\n" ); return 1; }
	const int nrays = argc > 2 ? atoi( argv[2] ) : 64000, refill = argc > 3 ? atoi( argv[3] ) : 48, leafBatch = argc > 4 ? atoi( argv[4] ) : 8;
	Model m;
	FILE* f = std::fopen( argv[1], "rb" );
	if (!f) return 1;
	std::fseek( f, 0, SEEK_END );
	const long bytes = std::ftell( f );
	std::fseek( f, 0, SEEK_SET );
	m.tv.resize( bytes / 4 );
	if (std::fread( m.tv.data(), 4, m.tv.size(), f ) != m.tv.size()) return 1;
	std::fclose( f );
	const size_t N = m.tv.size() / 9;
	std::vector<Aabb> prims( N );
	for (size_t i = 0; i < N; i++)
		for (int k = 0; k < 3; k++)
		{
			const float* v = &m.tv[i * 9];
			prims[i].lo[k] = std::fmin( std::fmin( v[k], v[3 + k] ), v[6 + k] );
			prims[i].hi[k] = std::fmax( std::fmax( v[k], v[3 + k] ), v[6 + k] );
		}
	BvhOutput out;
	BuildBvh2( prims, 1, 0, out, 1.0f, 0, m.tv.data(), 1e-3f, 1.0f, 0 );
	CollapseBvh4Sah( out.nodes.data(), out.nodes.size() / 16, m.n4, 0.4f, 0.5f, 1 );
	m.perm = out.perm;
	/* bounce stand-ins: random points on random triangles, cosine directions about the (random-sided) normal */
	std::mt19937 rng( 1234 );
	std::uniform_real_distribution<float> U( 0.0f, 1.0f );
	std::vector<Ray> rays;
	for (int i = 0; i < nrays; i++)
	{
		const uint32_t t = (uint32_t)(U( rng ) * N) % N;
		const float* v = &m.tv[(size_t)t * 9];
		float a = U( rng ), b = U( rng );
		if (a + b > 1) a = 1 - a, b = 1 - b;
		const V3 v0 = { v[0], v[1], v[2] }, e1 = sub( { v[3], v[4], v[5] }, v0 ), e2 = sub( { v[6], v[7], v[8] }, v0 );
		V3 n = norm( cross( e1, e2 ) );
		if (U( rng ) < 0.5f) n = { -n.x, -n.y, -n.z };
		const V3 o = { v0.x + a * e1.x + b * e2.x + n.x * 1e-4f, v0.y + a * e1.y + b * e2.y + n.y * 1e-4f, v0.z + a * e1.z + b * e2.z + n.z * 1e-4f };
		const V3 tt = std::fabs( n.x ) > 0.9f ? V3{ 0, 1, 0 } : V3{ 1, 0, 0 };
		const V3 T = norm( cross( n, tt ) ), B = cross( n, T );
		const float r1 = U( rng ), r2 = U( rng ), r = std::sqrt( r1 ), ph = 6.2831853f * r2, cz = std::sqrt( 1 - r1 );
		const V3 d = norm( { T.x * r * std::cos( ph ) + B.x * r * std::sin( ph ) + n.x * cz, T.y * r * std::cos( ph ) + B.y * r * std::sin( ph ) + n.y * cz,
			T.z * r * std::cos( ph ) + B.z * r * std::sin( ph ) + n.z * cz } );
		rays.push_back( { o, d, { 1.0f / d.x, 1.0f / d.y, 1.0f / d.z } } );
	}
	const char* names[3] = { "base", "pop-through", "slot2" };
	for (int v = 0; v < 3; v++)
	{
		const Counts c = simulate( m, rays, v, refill, leafBatch );
		std::printf( "{\"variant\": \"%s\", \"rays\": %d, \"refill\": %d, \"leafBatch\": %d, \"iters_per_ray\": %.3f, \"active_lanes\": %.1f, "
			"\"node_iter_frac\": %.3f, \"node_lanes\": %.1f, \"leaf_passes_per_ray\": %.3f, \"leaf_lanes\": %.1f, \"refills_per_ray\": %.4f, "
			"\"valu_per_ray\": %.1f, \"lane_util\": %.3f}\n", names[v], nrays, refill, leafBatch, c.iters * 64 / nrays, c.active / c.iters,
			c.nodeIters / c.iters, c.nodeLanes / c.nodeIters, c.leafPasses * 64 / nrays, c.leafLanes / c.leafPasses, c.refills * 64 / nrays,
			c.valu * 64 / nrays, c.valuLanes / c.valu / 64 );
	}
	return 0;
}
