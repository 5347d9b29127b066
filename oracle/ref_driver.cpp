/* ref_driver.cpp - TEST INFRASTRUCTURE: a thin extern "C" driver around the reference CPU traversal
   (RenderCore_Bart: BVH2 build bvh.cpp:57-256, recursive traversal bvh.cpp:258-302, Möller–Trumbore
   common.h:19-50), compiled from the sources under /root/reference by oracle/Makefile.ref into
   oracle/_ref/libbart_ref.so.  Used to pin the oracle's traversal (tests/test_oracle_ref.py) and as
   the "reference" CPU baseline in bench.py.  No reference source is copied: this file only calls it.
*/
#include "core_settings.h"   /* RenderCore_Bart/core_settings.h (reference) */

#include <thread>
#include <vector>

using namespace lh2core;

struct BartScene { Mesh* mesh; };

extern "C" {

/* tris: CoreTri records (176 B each); builds the BVH exactly as RenderCore_Bart::SetGeometry does
   (RenderCore_Bart/rendercore.cpp:47-79) */
__attribute__( (visibility( "default" )) ) void* bart_build( const void* tris, int T )
{
	const CoreTri* tri = (const CoreTri*)tris;
	Mesh* mesh = new Mesh( 3 * T, T );
	mesh->bvh = new BVH2( mesh );
	mesh->aabb_min_bound = make_float3( FLT_MAX );
	mesh->aabb_max_bound = make_float3( -FLT_MAX );
	for (int i = 0; i < T; i++)
	{
		mesh->triangles[i] = tri[i];
		mesh->tri_centers[i] = (tri[i].vertex0 + tri[i].vertex1 + tri[i].vertex2) / 3.0f;
		mesh->tri_min_bounds[i] = fminf( fminf( tri[i].vertex0, tri[i].vertex1 ), tri[i].vertex2 );
		mesh->tri_max_bounds[i] = fmaxf( fmaxf( tri[i].vertex0, tri[i].vertex1 ), tri[i].vertex2 );
		mesh->aabb_min_bound = fminf( mesh->aabb_min_bound, mesh->tri_min_bounds[i] );
		mesh->aabb_max_bound = fmaxf( mesh->aabb_max_bound, mesh->tri_max_bounds[i] );
	}
	mesh->bvh->Rebuild();
	BartScene* s = new BartScene;
	s->mesh = mesh;
	return s;
}

__attribute__( (visibility( "default" )) ) void bart_free( void* scene )
{
	BartScene* s = (BartScene*)scene;
	delete s->mesh;
	delete s;
}

/* closest hit of n rays (origin xyz, direction xyz); out4 = {t (FLT_MAX on miss), material, Nx.. }
   as floats: {t, N.x, N.y, N.z}; visits = node visit counts (Bart's debug counter) */
__attribute__( (visibility( "default" )) ) void bart_trace( void* scene, const float* org3, const float* dir3, int n, float* out4,
	int* visits, int threads )
{
	BartScene* s = (BartScene*)scene;
	if (threads < 1) threads = 1;
	auto work = [&]( int i0, int i1 ) {
		for (int i = i0; i < i1; i++)
		{
			Ray ray( make_float3( org3[i * 3], org3[i * 3 + 1], org3[i * 3 + 2] ), make_float3( dir3[i * 3], dir3[i * 3 + 1], dir3[i * 3 + 2] ) );
			int material = -1, c = 0;
			float3 N = make_float3( 0, 0, 0 );
			float t = FLT_MAX;
			s->mesh->bvh->Traverse( ray, material, N, t, 0, visits ? &c : nullptr );
			out4[i * 4 + 0] = t, out4[i * 4 + 1] = N.x, out4[i * 4 + 2] = N.y, out4[i * 4 + 3] = N.z;
			if (visits) visits[i] = c;
		}
	};
	if (threads == 1) { work( 0, n ); return; }
	std::vector<std::thread> th;
	for (int k = 0; k < threads; k++) th.emplace_back( work, (int)((long long)n * k / threads), (int)((long long)n * (k + 1) / threads) );
	for (auto& t : th) t.join();
}

}  // extern "C"
