/* bvh_width.cpp - host-side study (tools only): node steps per ray of the core's BLAS collapsed to BVH width
   K = 2, 4, 6, 8 (greedy surface-area collapse of the same SBVH BVH2, as CollapseBvh4 does for K = 4), traced
   nearest-first with the core's box test.  Reports per width the mean / p50 / p99 / max node steps and leaf
   visits of bounce stand-in rays (random surface points, cosine directions) and camera rays: the dependent
   chain that sets a launch's tail is the per-ray step count.
   Build: g++ -O2 -std=c++17 -pthread tools/bvh_width.cpp lighthouse2_amd/csrc/bvh_build.cpp -o /tmp/bvh_width
   Run:   /tmp/bvh_width tris.bin [spatialAlpha budget] [--camera px py pz tx ty tz] */
#include "../lighthouse2_amd/csrc/bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

using namespace lh2;

namespace {
struct V3 { float x, y, z; };
V3 sub( V3 a, V3 b ) { return { a.x - b.x, a.y - b.y, a.z - b.z }; }
V3 cross( V3 a, V3 b ) { return { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x }; }
float dot( V3 a, V3 b ) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 norm( V3 a ) { const float l = std::sqrt( dot( a, a ) ); return { a.x / l, a.y / l, a.z / l }; }

struct E { float lo[3], hi[3]; int ref; };
struct WNode { std::vector<E> c; };

struct Wide
{
	std::vector<WNode> nodes;
	const float* n2;
	int children( int k, E* out ) const
	{
		const float* n = n2 + (size_t)k * 16;
		int refs[2];
		memcpy( refs, n + 12, 8 );
		int m = 0;
		for (int c = 0; c < 2; c++)
		{
			E e;
			e.lo[0] = n[c * 4 + 0], e.hi[0] = n[c * 4 + 1], e.lo[1] = n[c * 4 + 2], e.hi[1] = n[c * 4 + 3];
			e.lo[2] = n[8 + c * 2], e.hi[2] = n[9 + c * 2], e.ref = refs[c];
			if (e.lo[0] == e.lo[0]) out[m++] = e;
		}
		return m;
	}
	static float area( const E& e )
	{
		const float dx = std::max( 0.0f, e.hi[0] - e.lo[0] ), dy = std::max( 0.0f, e.hi[1] - e.lo[1] ), dz = std::max( 0.0f, e.hi[2] - e.lo[2] );
		return dx * dy + dy * dz + dz * dx;
	}
	void build( const float* nodes2, int K )
	{
		n2 = nodes2;
		nodes.clear();
		nodes.push_back( {} );
		struct It { int n2, w; };
		std::vector<It> q{ { 0, 0 } };
		for (size_t qi = 0; qi < q.size(); qi++)
		{
			E list[16];
			int n = children( q[qi].n2, list );
			while (n < K)
			{
				int best = -1;
				float bA = -1;
				for (int i = 0; i < n; i++) if (list[i].ref >= 0 && area( list[i] ) > bA) best = i, bA = area( list[i] );
				if (best < 0) break;
				E c[2];
				const int m = children( list[best].ref, c );
				if (m == 0) { list[best] = list[--n]; continue; }
				list[best] = c[0];
				if (m == 2) list[n++] = c[1];
			}
			const int w = q[qi].w;
			for (int i = 0; i < n; i++)
			{
				E e = list[i];
				if (e.ref >= 0)
				{
					const int child = (int)nodes.size();
					nodes.push_back( {} );
					q.push_back( { e.ref, child } );
					e.ref = child;
				}
				nodes[w].c.push_back( e );
			}
		}
	}
};

struct Stats { std::vector<int> steps, leaves; double tris = 0; };

struct Tracer
{
	const Wide* W;
	const std::vector<float>* tv;
	const std::vector<uint32_t>* perm;
	bool isect( uint32_t t, V3 o, V3 d, float& tb ) const
	{
		const float* v = &(*tv)[(size_t)t * 9];
		const V3 v0 = { v[0], v[1], v[2] }, e1 = sub( { v[3], v[4], v[5] }, v0 ), e2 = sub( { v[6], v[7], v[8] }, v0 );
		const V3 p = cross( d, e2 );
		const float det = dot( e1, p );
		if (std::fabs( det ) < 1e-12f) return false;
		const float inv = 1.0f / det;
		const V3 s = sub( o, v0 );
		const float u = dot( s, p ) * inv;
		if (u < 0 || u > 1) return false;
		const V3 qq = cross( s, e1 );
		const float w = dot( d, qq ) * inv;
		if (w < 0 || u + w > 1) return false;
		const float tt = dot( e2, qq ) * inv;
		if (tt > 1e-4f && tt < tb) { tb = tt; return true; }
		return false;
	}
	void trace( V3 o, V3 d, Stats& st ) const
	{
		const V3 id = { 1.0f / d.x, 1.0f / d.y, 1.0f / d.z };
		float tb = 1e30f;
		std::vector<std::pair<float, int>> stack;
		int steps = 0, leaves = 0;
		stack.push_back( { 0.0f, 0 } );
		while (!stack.empty())
		{
			const auto [tn0, ref] = stack.back();
			stack.pop_back();
			if (tn0 > tb) continue;   /* t-culled pop (no step) */
			if (ref >= 0)
			{
				steps++;
				std::vector<std::pair<float, int>> hit;
				for (const E& e : W->nodes[ref].c)
				{
					float n = 0, f = 1e30f;
					const float oo[3] = { o.x, o.y, o.z }, ii[3] = { id.x, id.y, id.z };
					for (int k = 0; k < 3; k++)
					{
						const float a = (e.lo[k] - oo[k]) * ii[k], b = (e.hi[k] - oo[k]) * ii[k];
						n = std::fmax( n, std::fmin( a, b ) ), f = std::fmin( f, std::fmax( a, b ) );
					}
					if (n <= f * 1.00001f && n <= tb) hit.push_back( { n, e.ref } );
				}
				std::sort( hit.begin(), hit.end(), []( auto& a, auto& b ) { return a.first > b.first; } );
				for (auto& h : hit) stack.push_back( h );
			}
			else
			{
				leaves++;
				const uint32_t first = (uint32_t)(~ref) >> 4;
				const int cnt = (int)((uint32_t)(~ref) & 15u) + 1;
				for (int k = 0; k < cnt; k++) { st.tris++; isect( (*perm)[first + k], o, d, tb ); }
			}
		}
		st.steps.push_back( steps ), st.leaves.push_back( leaves );
	}
};

double pct( std::vector<int> v, double p ) { std::sort( v.begin(), v.end() ); return v.empty() ? 0 : v[(size_t)std::min( v.size() - 1.0, p * v.size() )]; }
double mean( const std::vector<int>& v ) { double s = 0; for (int x : v) s += x; return v.empty() ? 0 : s / v.size(); }
}  // namespace

int main( int argc, char** argv )
{
	if (argc < 2) return 1;
	float alpha = argc > 2 ? (float)atof( argv[2] ) : 1e-5f, budget = argc > 3 ? (float)atof( argv[3] ) : 1.0f;
	V3 cp = { 0, 0, -12 }, ct = { 0, 0, 1 };
	for (int i = 1; i + 6 < argc; i++) if (!strcmp( argv[i], "--camera" ))
		cp = { (float)atof( argv[i + 1] ), (float)atof( argv[i + 2] ), (float)atof( argv[i + 3] ) }, ct = { (float)atof( argv[i + 4] ), (float)atof( argv[i + 5] ), (float)atof( argv[i + 6] ) };
	std::vector<float> tv;
	FILE* f = std::fopen( argv[1], "rb" );
	std::fseek( f, 0, SEEK_END );
	tv.resize( std::ftell( f ) / 4 );
	std::fseek( f, 0, SEEK_SET );
	if (std::fread( tv.data(), 4, tv.size(), f ) != tv.size()) return 1;
	std::fclose( f );
	const size_t N = tv.size() / 9;
	std::vector<Aabb> prims( N );
	for (size_t i = 0; i < N; i++)
		for (int k = 0; k < 3; k++)
			prims[i].lo[k] = std::fmin( std::fmin( tv[i * 9 + k], tv[i * 9 + 3 + k] ), tv[i * 9 + 6 + k] ),
			prims[i].hi[k] = std::fmax( std::fmax( tv[i * 9 + k], tv[i * 9 + 3 + k] ), tv[i * 9 + 6 + k] );
	BvhOutput out;
	BuildBvh2( prims, 1, 0, out, 1.0f, 0, alpha > 0 ? tv.data() : nullptr, alpha, budget );
	std::mt19937 rng( 1234 );
	std::uniform_real_distribution<float> U( 0.0f, 1.0f );
	std::vector<std::pair<V3, V3>> surf, cam;
	for (int i = 0; i < 40000; i++)
	{
		const uint32_t t = (uint32_t)(U( rng ) * N) % N;
		const float* v = &tv[(size_t)t * 9];
		float a = U( rng ), b = U( rng );
		if (a + b > 1) a = 1 - a, b = 1 - b;
		const V3 v0 = { v[0], v[1], v[2] }, e1 = sub( { v[3], v[4], v[5] }, v0 ), e2 = sub( { v[6], v[7], v[8] }, v0 );
		V3 n = norm( cross( e1, e2 ) );
		if (U( rng ) < 0.5f) n = { -n.x, -n.y, -n.z };
		const V3 o = { v0.x + a * e1.x + b * e2.x + n.x * 1e-4f, v0.y + a * e1.y + b * e2.y + n.y * 1e-4f, v0.z + a * e1.z + b * e2.z + n.z * 1e-4f };
		const V3 tt = std::fabs( n.x ) > 0.9f ? V3{ 0, 1, 0 } : V3{ 1, 0, 0 };
		const V3 T = norm( cross( n, tt ) ), B = cross( n, T );
		const float r1 = U( rng ), r2 = U( rng ), r = std::sqrt( r1 ), ph = 6.2831853f * r2, cz = std::sqrt( 1 - r1 );
		surf.push_back( { o, norm( { T.x * r * std::cos( ph ) + B.x * r * std::sin( ph ) + n.x * cz, T.y * r * std::cos( ph ) + B.y * r * std::sin( ph ) + n.y * cz,
			T.z * r * std::cos( ph ) + B.z * r * std::sin( ph ) + n.z * cz } ) } );
	}
	const V3 fw = norm( ct ), rt = norm( cross( { 0, 1, 0 }, fw ) ), up = cross( fw, rt );
	const float th = std::tan( 40.0f * 3.14159265f / 360.0f ), aspect = 16.0f / 9.0f;
	for (int y = 0; y < 144; y++)
		for (int x = 0; x < 256; x++)
		{
			const float sx = ((x + 0.5f) / 256.0f * 2 - 1) * th * aspect, sy = ((y + 0.5f) / 144.0f * 2 - 1) * th;
			cam.push_back( { cp, norm( { fw.x + sx * rt.x + sy * up.x, fw.y + sx * rt.y + sy * up.y, fw.z + sx * rt.z + sy * up.z } ) } );
		}
	for (int K : { 2, 4, 6, 8 })
	{
		Wide W;
		W.build( out.nodes.data(), K );
		Tracer tr{ &W, &tv, &out.perm };
		Stats ss, sc;
		for (auto& r : surf) tr.trace( r.first, r.second, ss );
		for (auto& r : cam) tr.trace( r.first, r.second, sc );
		std::printf( "{\"K\": %d, \"nodes\": %zu, \"surface\": {\"steps\": %.2f, \"p50\": %.0f, \"p99\": %.0f, \"max\": %.0f, \"leaves\": %.2f, \"tris\": %.2f, "
			"\"iters_p99\": %.0f, \"iters_max\": %.0f}, \"camera\": {\"steps\": %.2f, \"p99\": %.0f, \"max\": %.0f, \"leaves\": %.2f}}\n",
			K, W.nodes.size(), mean( ss.steps ), pct( ss.steps, 0.5 ), pct( ss.steps, 0.99 ), pct( ss.steps, 1.0 ), mean( ss.leaves ), ss.tris / surf.size(),
			[&] { std::vector<int> it( ss.steps.size() ); for (size_t i = 0; i < it.size(); i++) it[i] = ss.steps[i] + ss.leaves[i]; return pct( it, 0.99 ); }(),
			[&] { std::vector<int> it( ss.steps.size() ); for (size_t i = 0; i < it.size(); i++) it[i] = ss.steps[i] + ss.leaves[i]; return pct( it, 1.0 ); }(),
			mean( sc.steps ), pct( sc.steps, 0.99 ), pct( sc.steps, 1.0 ), mean( sc.leaves ) );
		std::fflush( stdout );
	}
	return 0;
}
