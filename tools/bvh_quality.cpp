/* bvh_quality.cpp - host-side traversal cost of the core's BVH4 (tools only): builds the BLAS the way
   RenderCore::SetGeometry does (bvh_build.cpp: binned SAH, optionally spatial splits, greedy BVH4
   collapse), then traces sample rays with a nearest-first BVH4 walk and reports node steps and
   triangle tests per ray - the work the GPU traversal loop does per ray.
     rays "camera": a pinhole camera grid; "surface": from random points on random triangles, cosine
     distributed about the normal (a stand-in for the bounce rays).
   Build: g++ -O2 -std=c++17 -pthread tools/bvh_quality.cpp lighthouse2_amd/csrc/bvh_build.cpp -o /tmp/bvh_quality
   Run:   /tmp/bvh_quality tris.bin [alpha budget maxLeaf]   (tris.bin: float32 v0 v1 v2 per triangle)
          camera: pos (0, 0, -12), looking +z, vertical FOV 40, 16:9 (config 2), or --camera px py pz tx ty tz */
#include "../lighthouse2_amd/csrc/bvh_build.h"

#include <algorithm>
#include <chrono>
#include <cmath>
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

struct Stats { double nodes = 0, tris = 0, leaves = 0, hits = 0; int rays = 0; std::vector<int> per; std::vector<float> chord; };

struct Scene
{
	std::vector<float> tv;          /* 9 per triangle */
	std::vector<float> n4;          /* BVH4 nodes */
	std::vector<uint32_t> perm;

	bool intersect( uint32_t t, V3 o, V3 d, float& tb ) const
	{
		const float* v = &tv[(size_t)t * 9];
		const V3 v0 = { v[0], v[1], v[2] }, e1 = sub( { v[3], v[4], v[5] }, v0 ), e2 = sub( { v[6], v[7], v[8] }, v0 );
		const V3 p = cross( d, e2 );
		const float det = dot( e1, p );
		if (std::fabs( det ) < 1e-12f) return false;
		const float inv = 1.0f / det;
		const V3 s = sub( o, v0 );
		const float u = dot( s, p ) * inv;
		if (u < 0 || u > 1) return false;
		const V3 q = cross( s, e1 );
		const float w = dot( d, q ) * inv;
		if (w < 0 || u + w > 1) return false;
		const float tt = dot( e2, q ) * inv;
		if (tt > 1e-4f && tt < tb) { tb = tt; return true; }
		return false;
	}
	void trace( V3 o, V3 d, Stats& st, std::vector<int>* visited = nullptr ) const
	{
		const V3 id = { 1.0f / d.x, 1.0f / d.y, 1.0f / d.z };
		float tb = 1e30f;
		int stack[256], sp = 0, node = 0, steps = 0;
		bool hit = false;
		while (true)
		{
			if (node >= 0)
			{
				st.nodes++, steps++;
				if (visited) visited->push_back( node );
				const float* q = &n4[(size_t)node * 32];
				const int* refs = (const int*)(q + 24);
				float tn[4]; int order[4], nh = 0;
				for (int c = 0; c < 4; c++)
				{
					/* planes of four: lo.x, hi.x, lo.y, hi.y, lo.z, hi.z (lh2_device.h) */
					const float lx = q[c], hx = q[4 + c], ly = q[8 + c], hy = q[12 + c], lz = q[16 + c], hz = q[20 + c];
					if (!(lx == lx)) continue;
					const float ax = (lx - o.x) * id.x, bx = (hx - o.x) * id.x, ay = (ly - o.y) * id.y, by = (hy - o.y) * id.y;
					const float az = (lz - o.z) * id.z, bz = (hz - o.z) * id.z;
					const float n = std::fmax( std::fmax( std::fmin( ax, bx ), std::fmin( ay, by ) ), std::fmax( std::fmin( az, bz ), 0.0f ) );
					const float f = std::fmin( std::fmin( std::fmax( ax, bx ), std::fmax( ay, by ) ), std::fmax( az, bz ) );
					if (n <= f * 1.00001f && n <= tb) { tn[nh] = n, order[nh] = refs[c]; nh++; }
				}
				for (int i = 1; i < nh; i++)
					for (int k = i; k > 0 && tn[k] < tn[k - 1]; k--) std::swap( tn[k], tn[k - 1] ), std::swap( order[k], order[k - 1] );
				for (int i = nh - 1; i >= 1; i--) stack[sp++] = order[i];
				if (nh) { node = order[0]; continue; }
			}
			else
			{
				const uint32_t first = (uint32_t)(~node) >> 4;
				const int cnt = (int)((uint32_t)(~node) & 15u) + 1;
				st.leaves++, steps++;
				for (int k = 0; k < cnt; k++) { st.tris++; hit |= intersect( perm[first + k], o, d, tb ); }
			}
			if (sp == 0) break;
			node = stack[--sp];
		}
		st.hits += hit;
		st.rays++;
		st.per.push_back( steps );
	}
};

}  // namespace

int main( int argc, char** argv )
{
	if (argc < 2) { std::fprintf( stderr, "usage: bvh_quality tris.bin [alpha budget maxLeaf]\n" ); return 1; }
	const float alpha = argc > 2 ? (float)atof( argv[2] ) : 0.0f, budget = argc > 3 ? (float)atof( argv[3] ) : 0.3f;
	const int maxLeaf = argc > 4 ? atoi( argv[4] ) : 1;
	Scene sc;
	FILE* f = std::fopen( argv[1], "rb" );
	if (!f) return 1;
	std::fseek( f, 0, SEEK_END );
	const long bytes = std::ftell( f );
	std::fseek( f, 0, SEEK_SET );
	sc.tv.resize( bytes / 4 );
	if (std::fread( sc.tv.data(), 4, sc.tv.size(), f ) != sc.tv.size()) return 1;
	std::fclose( f );
	const size_t N = sc.tv.size() / 9;
	std::vector<Aabb> prims( N );
	for (size_t i = 0; i < N; i++)
		for (int k = 0; k < 3; k++)
		{
			const float* v = &sc.tv[i * 9];
			prims[i].lo[k] = std::fmin( std::fmin( v[k], v[3 + k] ), v[6 + k] );
			prims[i].hi[k] = std::fmax( std::fmax( v[k], v[3 + k] ), v[6 + k] );
		}
	const auto t0 = std::chrono::steady_clock::now();
	BvhOutput out;
	const float ctrav = getenv( "CTRAV" ) ? (float)atof( getenv( "CTRAV" ) ) : 1.0f;
	const int minRefs = std::getenv( "LH2_MINREFS" ) ? atoi( std::getenv( "LH2_MINREFS" ) ) : 0;   /* bvhSpatialMinRefs */
	const int threads = std::getenv( "LH2_THREADS" ) ? atoi( std::getenv( "LH2_THREADS" ) ) : 0;
	BuildBvh2( prims, maxLeaf, threads, out, ctrav, 0, alpha > 0 ? sc.tv.data() : nullptr, alpha, budget, minRefs );
	const double buildS = std::chrono::duration<double>( std::chrono::steady_clock::now() - t0 ).count();
	const float cLeaf = argc > 5 ? (float)atof( argv[5] ) : -1.0f, cTri = argc > 6 ? (float)atof( argv[6] ) : 0.5f;
	const int mlt = argc > 7 ? atoi( argv[7] ) : 1;
	const int depth4 = cLeaf < 0 ? CollapseBvh4( out.nodes.data(), out.nodes.size() / 16, sc.n4 )
		: CollapseBvh4Sah( out.nodes.data(), out.nodes.size() / 16, sc.n4, cLeaf, cTri, mlt );
	sc.perm = out.perm;
	/* rays */
	std::mt19937 rng( 1234 );
	std::uniform_real_distribution<float> U( 0.0f, 1.0f );
	Stats cam, surf;
	const V3 cp = { 0, 0, -12 };
	const float th = std::tan( 40.0f * 3.14159265f / 360.0f ), aspect = 16.0f / 9.0f;
	for (int y = 0; y < 144; y++)
		for (int x = 0; x < 256; x++)
		{
			const float sx = ((x + 0.5f) / 256.0f * 2 - 1) * th * aspect, sy = ((y + 0.5f) / 144.0f * 2 - 1) * th;
			sc.trace( cp, norm( { sx, sy, 1.0f } ), cam );
		}
	for (int i = 0; i < 40000; i++)
	{
		const uint32_t t = (uint32_t)(U( rng ) * N) % N;
		const float* v = &sc.tv[(size_t)t * 9];
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
		sc.trace( o, d, surf );
		/* the ray's chord through the scene box (a predictor of its traversal cost) */
		float t1 = 1e30f;
		const float lo[3] = { -5.3f, -5.3f, -5.3f }, hi[3] = { 5.3f, 5.3f, 5.3f }, oo[3] = { o.x, o.y, o.z }, dd[3] = { d.x, d.y, d.z };
		for (int k = 0; k < 3; k++) t1 = std::fmin( t1, std::fmax( (lo[k] - oo[k]) / dd[k], (hi[k] - oo[k]) / dd[k] ) );
		surf.chord.push_back( t1 );
	}
	std::printf( "{\"tris\": %zu, \"alpha\": %g, \"budget\": %g, \"maxLeaf\": %d, \"refs\": %zu, \"nodes2\": %zu, \"nodes4\": %zu, \"depth2\": %d, "
		"\"depth4\": %d, \"sah\": %.3f, \"build_s\": %.2f, \"camera\": {\"nodes\": %.2f, \"leaves\": %.2f, \"tris\": %.2f, \"hit\": %.3f}, "
		"\"surface\": {\"nodes\": %.2f, \"leaves\": %.2f, \"tris\": %.2f, \"hit\": %.3f}, \"valu_model\": %.0f}\n",
		N, alpha, budget, maxLeaf, out.perm.size(), out.nodes.size() / 16, sc.n4.size() / 32, out.maxDepth, depth4, out.sah, buildS,
		cam.nodes / cam.rays, cam.leaves / cam.rays, cam.tris / cam.rays, cam.hits / cam.rays, surf.nodes / surf.rays, surf.leaves / surf.rays, surf.tris / surf.rays, surf.hits / surf.rays,
		(175.0 * surf.nodes + 66.0 * surf.leaves + 86.0 * surf.tris) / surf.rays );
	if (getenv( "TILES" ))
	{
		/* the config-2 frame's 8x8 primary-ray tiles: per tile, the union of the nodes its rays visit
		   (what a packet traverses) and the longest ray */
		const int W = 1920, H = 1080;
		std::vector<std::pair<int, int>> cost;   /* (union, max steps) */
		Stats tmp;
		for (int ty = 0; ty < H / 8; ty++)
			for (int tx = 0; tx < W / 8; tx++)
			{
				std::vector<int> vis;
				int mx = 0;
				for (int y = ty * 8; y < ty * 8 + 8; y++)
					for (int x = tx * 8; x < tx * 8 + 8; x++)
					{
						const float sx = ((x + 0.5f) / W * 2 - 1) * th * aspect, sy = ((y + 0.5f) / H * 2 - 1) * th;
						const size_t before = vis.size();
						sc.trace( cp, norm( { sx, sy, 1.0f } ), tmp, &vis );
						mx = std::max( mx, (int)(vis.size() - before) );
					}
				std::sort( vis.begin(), vis.end() );
				const int uni = (int)(std::unique( vis.begin(), vis.end() ) - vis.begin());
				cost.push_back( { uni, mx } );
			}
		if (const char* out = getenv( "TILES_OUT" ))
			if (FILE* fo = std::fopen( out, "wb" ))
			{
				for (auto& c : cost) { const int32_t v = c.first; std::fwrite( &v, 4, 1, fo ); }
				std::fclose( fo );
			}
		std::vector<int> u, m;
		for (auto& c : cost) u.push_back( c.first ), m.push_back( c.second );
		std::sort( u.begin(), u.end() ), std::sort( m.begin(), m.end() );
		const size_t n = u.size();
		double su = 0; for (int x : u) su += x;
		std::printf( "tiles %zu: union nodes p50 %d p90 %d p99 %d max %d (sum %.0f, top 1%% share %.3f); longest ray p50 %d p99 %d max %d\n", n,
			u[n / 2], u[n * 9 / 10], u[n * 99 / 100], u.back(), su, [&]() { double t = 0; for (size_t i = n * 99 / 100; i < n; i++) t += u[i]; return t / su; }(),
			m[n / 2], m[n * 99 / 100], m.back() );
	}
	if (getenv( "DIST" ))
	{
		std::vector<std::pair<float, int>> cs;
		for (size_t i = 0; i < surf.per.size(); i++) cs.push_back( { surf.chord[i], surf.per[i] } );
		std::sort( cs.begin(), cs.end() );
		for (int dcl = 0; dcl < 10; dcl++)
		{
			std::vector<int> v;
			for (size_t i = cs.size() * dcl / 10; i < cs.size() * (dcl + 1) / 10; i++) v.push_back( cs[i].second );
			std::sort( v.begin(), v.end() );
			double m = 0; for (int x : v) m += x;
			std::printf( "chord decile %d (%.2f..): mean %.1f p90 %d p99 %d max %d\n", dcl, cs[cs.size() * dcl / 10].first, m / v.size(), v[v.size() * 9 / 10], v[v.size() * 99 / 100], v.back() );
		}
		std::sort( surf.per.begin(), surf.per.end() );
		const size_t n = surf.per.size();
		std::printf( "surface iterations per ray: p50 %d p90 %d p99 %d p99.9 %d max %d\n", surf.per[n / 2], surf.per[n * 9 / 10], surf.per[n * 99 / 100], surf.per[n * 999 / 1000], surf.per.back() );
	}
	return 0;
}
