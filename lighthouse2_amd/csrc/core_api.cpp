/* core_api.cpp - the drop-in boundary: CoreAPI_Base implementation, CreateCore / DestroyCore,
   and the flat extern "C" mirror declared in include/lh2_rendercore.h.

   Reference: RenderCore_OptixPrime_B/core_api.cpp:20-122 and core_api.h:26-64.  CreateCore is a
   process singleton that calls Init(); the loader (core_api_base.cpp:129) calls Init() again, so
   Init is idempotent.  gladLoadGL() (core_api.cpp:23) is not called: this core is headless and
   never touches OpenGL (GLTexture::ID is ignored; the frame is read back via lh2_core_get_frame).
*/
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/lh2_core_api.hpp"
#include "../../include/lh2_rendercore.h"
#include "rendercore.h"

#define LH2_EXPORT __attribute__( (visibility( "default" )) )

static thread_local std::string g_lastError;

namespace lh2 {

class CoreAPI final : public lh2abi::CoreAPI_Base
{
public:
	bool throwErrors = false;   /* flat C-ABI instances report errors instead of exiting */
	RenderCore* core = nullptr;

	template <class F> void guard( F&& f )
	{
		try { f(); }
		catch (const std::exception& e)
		{
			if (throwErrors) throw;
			/* reference FatalError on Linux: print, then exit(0) (platform/system.cpp:221-236) */
			fprintf( stderr, "RenderCore_MI355X fatal error: %s\n", e.what() );
			exit( 0 );
		}
	}
	lh2_CoreStats GetCoreStats() override { lh2_CoreStats s{}; guard( [&] { s = core->GetCoreStats(); } ); return s; }
	void Init() override { guard( [&] { if (!core) { core = new RenderCore(); core->Init(); } } ); }
	void SetProbePos( const lh2_int2 pos ) override { core->SetProbePos( pos.x, pos.y ); }
	void SetTarget( lh2abi::GLTextureView* t, const uint32_t spp ) override
	{
		/* a GL texture (ID != 0, GL context current) receives every finalized frame through HIP-GL
		   interop, as InteropTexture does for the CUDA cores (interoptexture.cpp:51-71) */
		guard( [&] { core->SetTarget( t->width, t->height, spp ); core->SetInteropTexture( t->ID ); } );
	}
	void Setting( const char* name, float value ) override { guard( [&] { core->Setting( name, value ); } ); }
	void Render( const lh2_ViewPyramid& view, const int converge ) override { guard( [&] { core->Render( view, converge ); } ); }
	void Shutdown() override { guard( [&] { if (core) { core->Shutdown(); delete core; core = nullptr; } } ); }
	void SetTextures( const lh2_CoreTexDesc* tex, const int n ) override { guard( [&] { core->SetTextures( tex, n ); } ); }
	void SetMaterials( lh2_CoreMaterial* mat, const int n ) override { guard( [&] { core->SetMaterials( mat, n ); } ); }
	void SetLights( const lh2_CoreLightTri* a, const int na, const lh2_CorePointLight* p, const int np, const lh2_CoreSpotLight* s, const int ns,
		const lh2_CoreDirectionalLight* d, const int nd ) override
	{
		guard( [&] { core->SetLights( a, na, p, np, s, ns, d, nd ); } );
	}
	void SetSkyData( const lh2_float3* px, const uint32_t w, const uint32_t h, const lh2_mat4& ) override { guard( [&] { core->SetSkyData( (const float*)px, w, h ); } ); }
	void SetGeometry( const int meshIdx, const lh2_float4* v, const int vc, const int tc, const lh2_CoreTri* t, const uint32_t* alpha ) override
	{
		guard( [&] { core->SetGeometry( meshIdx, (const float*)v, vc, tc, t, alpha ); } );
	}
	void SetInstance( const int idx, const int mesh, const lh2_mat4& T ) override { guard( [&] { core->SetInstance( idx, mesh, T.cell ); } ); }
	void UpdateToplevel() override { guard( [&] { core->UpdateToplevel(); } ); }
};

}  // namespace lh2

using lh2::CoreAPI;

static lh2abi::CoreAPI_Base* coreInstance = nullptr;

extern "C" LH2_EXPORT lh2abi::CoreAPI_Base* CreateCore()   /* core_api.cpp:20-27 */
{
	if (coreInstance) { fprintf( stderr, "CreateCore: core already exists\n" ); exit( 0 ); }
	coreInstance = new CoreAPI();
	coreInstance->Init();
	return coreInstance;
}

extern "C" LH2_EXPORT void DestroyCore()   /* core_api.cpp:29-34 */
{
	delete static_cast<CoreAPI*>( coreInstance );
	coreInstance = nullptr;
}

/* ------------------------------------------------------------------------------------------ */
/* flat C mirror: every call goes through the CoreAPI_Base vtable                              */
/* ------------------------------------------------------------------------------------------ */
template <class F> static int wrap( F&& f )
{
	try { f(); return 0; }
	catch (const std::exception& e) { g_lastError = e.what(); return -1; }
	catch (...) { g_lastError = "unknown error"; return -1; }
}
static lh2abi::CoreAPI_Base* B( lh2_core c )
{
	if (!c) throw std::runtime_error( "null core handle" );
	return static_cast<lh2abi::CoreAPI_Base*>( c );
}
static lh2::RenderCore* R( lh2_core c )
{
	CoreAPI* api = static_cast<CoreAPI*>( B( c ) );
	if (!api->core) throw std::runtime_error( "core not initialised" );
	return api->core;
}

extern "C" {

LH2_EXPORT const char* lh2_version( void ) { return "RenderCore_MI355X 0.1 (gfx950)"; }
LH2_EXPORT const char* lh2_last_error( void ) { return g_lastError.c_str(); }
LH2_EXPORT int lh2_set_device( int device )
{
	return wrap( [&] { if (hipSetDevice( device ) != hipSuccess) throw std::runtime_error( "hipSetDevice failed" ); } );
}

LH2_EXPORT int lh2_core_new( lh2_core* out )
{
	return wrap( [&] {
		CoreAPI* api = new CoreAPI();
		api->throwErrors = true;
		try { static_cast<lh2abi::CoreAPI_Base*>( api )->Init(); }
		catch (...) { delete api; throw; }
		*out = static_cast<lh2abi::CoreAPI_Base*>( api );
	} );
}
LH2_EXPORT int lh2_core_delete( lh2_core c )
{
	return wrap( [&] { CoreAPI* api = static_cast<CoreAPI*>( B( c ) ); if (api->core) B( c )->Shutdown(); delete api; } );
}
LH2_EXPORT int lh2_core_init( lh2_core c ) { return wrap( [&] { B( c )->Init(); } ); }
LH2_EXPORT int lh2_core_get_stats( lh2_core c, lh2_CoreStats* out ) { return wrap( [&] { *out = B( c )->GetCoreStats(); } ); }
LH2_EXPORT int lh2_core_set_probe( lh2_core c, int x, int y ) { return wrap( [&] { lh2_int2 p; p.x = x, p.y = y; B( c )->SetProbePos( p ); } ); }
LH2_EXPORT int lh2_core_set_target( lh2_core c, uint32_t w, uint32_t h, uint32_t spp )
{
	return wrap( [&] { lh2abi::GLTextureView t{ 0, w, h }; B( c )->SetTarget( &t, spp ); } );
}
LH2_EXPORT int lh2_core_setting( lh2_core c, const char* name, float v ) { return wrap( [&] { B( c )->Setting( name, v ); } ); }
LH2_EXPORT int lh2_core_render( lh2_core c, const lh2_ViewPyramid* view, int converge ) { return wrap( [&] { B( c )->Render( *view, converge ); } ); }
LH2_EXPORT int lh2_core_shutdown( lh2_core c ) { return wrap( [&] { B( c )->Shutdown(); } ); }
LH2_EXPORT int lh2_core_set_textures( lh2_core c, const lh2_CoreTexDesc* t, int n ) { return wrap( [&] { B( c )->SetTextures( t, n ); } ); }
LH2_EXPORT int lh2_core_set_materials( lh2_core c, lh2_CoreMaterial* m, int n ) { return wrap( [&] { B( c )->SetMaterials( m, n ); } ); }
LH2_EXPORT int lh2_core_set_lights( lh2_core c, const lh2_CoreLightTri* a, int na, const lh2_CorePointLight* p, int np,
	const lh2_CoreSpotLight* s, int ns, const lh2_CoreDirectionalLight* d, int nd )
{
	return wrap( [&] { B( c )->SetLights( a, na, p, np, s, ns, d, nd ); } );
}
LH2_EXPORT int lh2_core_set_sky( lh2_core c, const float* rgb, uint32_t w, uint32_t h )
{
	return wrap( [&] { lh2_mat4 I{}; for (int i = 0; i < 16; i++) I.cell[i] = (i % 5 == 0) ? 1.0f : 0.0f; B( c )->SetSkyData( (const lh2_float3*)rgb, w, h, I ); } );
}
LH2_EXPORT int lh2_core_set_geometry( lh2_core c, int meshIdx, const float* v4, int vc, int tc, const lh2_CoreTri* t, const uint32_t* alpha )
{
	return wrap( [&] { B( c )->SetGeometry( meshIdx, (const lh2_float4*)v4, vc, tc, t, alpha ); } );
}
LH2_EXPORT int lh2_core_set_instance( lh2_core c, int idx, int mesh, const float* m16 )
{
	return wrap( [&] { lh2_mat4 M; if (m16) memcpy( M.cell, m16, 64 ); else for (int i = 0; i < 16; i++) M.cell[i] = (i % 5 == 0) ? 1.0f : 0.0f; B( c )->SetInstance( idx, mesh, M ); } );
}
LH2_EXPORT int lh2_core_update_toplevel( lh2_core c ) { return wrap( [&] { B( c )->UpdateToplevel(); } ); }

LH2_EXPORT int lh2_core_set_tile( lh2_core c, int y0, int y1 ) { return wrap( [&] { R( c )->SetTile( y0, y1 ); } ); }
LH2_EXPORT int lh2_core_set_tile_bands( lh2_core c, int rank, int nranks, int band )
{
	return wrap( [&] { if (nranks < 1 || rank < 0 || rank >= nranks || band < 1) throw std::runtime_error( "bad tile bands" ); R( c )->SetTileBands( rank, nranks, band ); } );
}
LH2_EXPORT int lh2_core_sync( lh2_core c ) { return wrap( [&] { R( c )->Synchronize(); } ); }
LH2_EXPORT int lh2_core_get_accumulator( lh2_core c, float* out ) { return wrap( [&] { R( c )->GetAccumulator( out ); } ); }
LH2_EXPORT int lh2_core_get_frame( lh2_core c, float* out ) { return wrap( [&] { R( c )->GetFrame( out ); } ); }
LH2_EXPORT int lh2_core_copy_accumulator_rows( lh2_core c, void* dst, int y0, int y1 ) { return wrap( [&] { R( c )->CopyAccumulatorRows( dst, y0, y1 ); } ); }
LH2_EXPORT int lh2_core_pack_tile( lh2_core c, void* dst ) { return wrap( [&] { R( c )->PackTile( dst ); } ); }
LH2_EXPORT int lh2_core_pack_tile_ordered( lh2_core c, void* dst, void* consumerStream ) { return wrap( [&] { R( c )->PackTile( dst, true, consumerStream ); } ); }
LH2_EXPORT int lh2_core_tile_rows( lh2_core c, int* rows ) { return wrap( [&] { *rows = R( c )->TileRows(); } ); }
LH2_EXPORT int lh2_core_stream( lh2_core c, void** stream ) { return wrap( [&] { *stream = (void*)R( c )->stream; } ); }
LH2_EXPORT int lh2_core_ray_counts( lh2_core c, uint32_t* out17 ) { return wrap( [&] { R( c )->GetRayCounts( out17 ); } ); }
LH2_EXPORT int lh2_core_trace_closest( lh2_core c, const float* o, const float* d, int n, uint32_t* h ) { return wrap( [&] { R( c )->TraceClosest( o, d, n, h ); } ); }
LH2_EXPORT int lh2_core_trace_any( lh2_core c, const float* o, const float* d, int n, uint32_t* m ) { return wrap( [&] { R( c )->TraceAny( o, d, n, m ); } ); }
LH2_EXPORT int lh2_core_trace_closest_device( lh2_core c, const void* o, const void* d, int n, void* h, int it, float* ms )
{
	return wrap( [&] { R( c )->TraceClosestDevice( o, d, n, h, it, ms ); } );
}
LH2_EXPORT int lh2_core_generate_eye_rays( lh2_core c, const lh2_ViewPyramid* v, uint32_t R0, int pass, float* o, float* d, float* s )
{
	return wrap( [&] { R( c )->GenerateEyeRays( *v, R0, pass, o, d, s ); } );
}
LH2_EXPORT int lh2_core_scene_info( lh2_core c, int* nodes, int* tris, int* depth, int* inst ) { return wrap( [&] { R( c )->SceneInfo( nodes, tris, depth, inst ); } ); }

LH2_EXPORT int lh2_xorshift_floats( uint32_t seed, float* out, uint64_t n )
{
	uint32_t s = seed;
	for (uint64_t i = 0; i < n; i++) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; out[i] = (float)s * 2.3283064365387e-10f; }
	return 0;
}

}  // extern "C"
