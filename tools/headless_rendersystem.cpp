/* headless_rendersystem.cpp - replay a recorded CoreAPI call stream through the RenderCore dll boundary.

   This is what an unchanged Lighthouse 2 RenderSystem does with a core (and nothing more):
     dlopen("libRenderCore_MI355X.so", RTLD_NOW | RTLD_GLOBAL)       RenderSystem/core_api_base.cpp:97-110
     dlsym("CreateCore") / dlsym("DestroyCore")                       core_api_base.cpp:124-127
     core->Init() (a second time; CreateCore already called it)       core_api_base.cpp:129
     SetTarget / SetMaterials / SetGeometry / SetInstance(-1 ends) /
     UpdateToplevel / SetLights / Setting / Render / GetCoreStats     rendersystem.cpp:22-301
   through the CoreAPI_Base vtable declared in include/lh2_core_api.hpp.  No Python, no torch and
   no flat C layer are involved; the only non-vtable call is the headless readback extension
   lh2_core_get_accumulator (the reference core would blit to a GL texture instead).

   The call stream comes from lighthouse2_amd/record.py (CallRecorder).

   Build:  g++ -O2 -std=c++17 -I include tools/headless_rendersystem.cpp -ldl -o build/headless_rendersystem
   Run:    build/headless_rendersystem <lib.so> <calls.bin> <accumulator.out> [--parse-only]
*/
#include <dlfcn.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "lh2_core_api.hpp"

using lh2abi::CoreAPI_Base;

namespace {

enum Op : uint32_t { SET_SKY = 1, SET_MATERIALS, SET_GEOMETRY, SET_INSTANCE, UPDATE_TOPLEVEL, SET_LIGHTS, SETTING, SET_TARGET, RENDER, SET_PROBE, SET_TEXTURES };

struct Reader
{
	const uint8_t* p; size_t n, off = 0;
	template <class T> T get() { T v; std::memcpy( &v, p + off, sizeof( T ) ); off += sizeof( T ); return v; }
	const uint8_t* take( size_t bytes ) { const uint8_t* q = p + off; off += bytes; return q; }
};

template <class T> std::vector<T> copy_array( Reader& r, size_t count )
{
	std::vector<T> v( count ? count : 1 );
	if (count) std::memcpy( v.data(), r.take( sizeof( T ) * count ), sizeof( T ) * count );
	return v;
}

int fail( const char* msg ) { std::fprintf( stderr, "headless_rendersystem: %s\n", msg ); return 1; }

}  // namespace

int main( int argc, char** argv )
{
	if (argc < 4) return fail( "usage: headless_rendersystem <lib.so> <calls.bin> <accumulator.out> [--parse-only]" );
	const bool parseOnly = argc > 4 && std::strcmp( argv[4], "--parse-only" ) == 0;
	FILE* f = std::fopen( argv[2], "rb" );
	if (!f) return fail( "cannot open call stream" );
	std::vector<uint8_t> buf;
	{
		uint8_t tmp[1 << 16];
		size_t got;
		while ((got = std::fread( tmp, 1, sizeof( tmp ), f )) > 0) buf.insert( buf.end(), tmp, tmp + got );
		std::fclose( f );
	}

	CoreAPI_Base* core = nullptr;
	void* lib = nullptr;
	void (*destroy)() = nullptr;
	int (*getAccumulator)( void*, float* ) = nullptr;
	if (!parseOnly)
	{
		lib = dlopen( argv[1], RTLD_NOW | RTLD_GLOBAL );
		if (!lib) return fail( dlerror() );
		auto create = (CoreAPI_Base * (*)()) dlsym( lib, "CreateCore" );
		destroy = (void (*)()) dlsym( lib, "DestroyCore" );
		getAccumulator = (int (*)( void*, float* )) dlsym( lib, "lh2_core_get_accumulator" );
		if (!create || !destroy) return fail( "CreateCore/DestroyCore not exported" );
		core = create();
		core->Init();   /* CreateCoreAPI calls Init again: must be idempotent */
	}

	Reader r{ buf.data(), buf.size() };
	uint32_t w = 0, h = 0;
	int calls = 0, frames = 0;
	while (r.off + 8 <= r.n)
	{
		const uint32_t op = r.get<uint32_t>(), bytes = r.get<uint32_t>();
		const size_t end = r.off + bytes;
		if (end > r.n) return fail( "truncated call stream" );
		calls++;
		switch (op)
		{
		case SET_TARGET:
		{
			lh2abi::GLTextureView t{ 0, r.get<uint32_t>(), r.get<uint32_t>() };
			const uint32_t spp = r.get<uint32_t>();
			w = t.width, h = t.height;
			if (core) core->SetTarget( &t, spp );
			break;
		}
		case SETTING:
		{
			char name[33] = {};
			std::memcpy( name, r.take( 32 ), 32 );
			const float v = r.get<float>();
			if (core) core->Setting( name, v );
			break;
		}
		case SET_PROBE:
		{
			lh2_int2 p; p.x = r.get<int>(), p.y = r.get<int>();
			if (core) core->SetProbePos( p );
			break;
		}
		case SET_TEXTURES:
		{
			/* per texture: width, height, flags, pixelCount, MIPlevels, storage, texel bytes, texels (record.py); the
			   descriptors point at this host's copies for the duration of the call (rendercore.cpp:276-347) */
			const int n = r.get<int>();
			std::vector<lh2_CoreTexDesc> d( n > 0 ? n : 1 );
			std::vector<std::vector<uint8_t>> texels( n > 0 ? n : 1 );
			for (int i = 0; i < n; i++)
			{
				d[i].width = r.get<uint32_t>(), d[i].height = r.get<uint32_t>(), d[i].flags = r.get<uint32_t>();
				d[i].pixelCount = r.get<uint32_t>(), d[i].MIPlevels = r.get<uint32_t>();
				d[i].storage = r.get<int32_t>();
				d[i].firstPixel = 0;
				const uint32_t bytes = r.get<uint32_t>();
				const uint8_t* src = r.take( bytes );
				texels[i].assign( src, src + bytes );
				d[i].idata = (void*)texels[i].data();
			}
			if (core) core->SetTextures( d.data(), n );
			break;
		}
		case SET_MATERIALS:
		{
			const int n = r.get<int>();
			auto m = copy_array<lh2_CoreMaterial>( r, n );
			if (core) core->SetMaterials( m.data(), n );
			break;
		}
		case SET_LIGHTS:
		{
			const int na = r.get<int>(), np = r.get<int>(), ns = r.get<int>(), nd = r.get<int>();
			auto a = copy_array<lh2_CoreLightTri>( r, na );
			auto p = copy_array<lh2_CorePointLight>( r, np );
			auto s = copy_array<lh2_CoreSpotLight>( r, ns );
			auto d = copy_array<lh2_CoreDirectionalLight>( r, nd );
			if (core) core->SetLights( a.data(), na, p.data(), np, s.data(), ns, d.data(), nd );
			break;
		}
		case SET_SKY:
		{
			const uint32_t sw = r.get<uint32_t>(), sh = r.get<uint32_t>();
			auto px = copy_array<lh2_float3>( r, (size_t)sw * sh );
			lh2_mat4 I{};
			for (int i = 0; i < 16; i++) I.cell[i] = (i % 5 == 0) ? 1.0f : 0.0f;
			if (core) core->SetSkyData( px.data(), sw, sh, I );
			break;
		}
		case SET_GEOMETRY:
		{
			const int idx = r.get<int>(), n = r.get<int>();
			auto verts = copy_array<lh2_float4>( r, (size_t)3 * n );
			auto tris = copy_array<lh2_CoreTri>( r, n );
			if (core) core->SetGeometry( idx, verts.data(), 3 * n, n, tris.data(), nullptr );
			break;
		}
		case SET_INSTANCE:
		{
			const int idx = r.get<int>(), mesh = r.get<int>();
			lh2_mat4 T;
			std::memcpy( &T, r.take( 64 ), 64 );
			if (core) core->SetInstance( idx, mesh, T );
			break;
		}
		case UPDATE_TOPLEVEL:
			if (core) core->UpdateToplevel();
			break;
		case RENDER:
		{
			lh2_ViewPyramid view;
			std::memcpy( &view, r.take( sizeof( view ) ), sizeof( view ) );
			const int converge = r.get<int>();
			if (core) core->Render( view, converge );
			frames++;
			break;
		}
		default: return fail( "unknown opcode" );
		}
		if (r.off != end) return fail( "payload size mismatch" );
	}
	if (parseOnly)
	{
		std::printf( "{\"calls\": %d, \"frames\": %d, \"width\": %u, \"height\": %u}\n", calls, frames, w, h );
		return 0;
	}
	const lh2_CoreStats st = core->GetCoreStats();   /* returned by value through the vtable */
	std::printf( "{\"calls\": %d, \"frames\": %d, \"primaryRayCount\": %u, \"bounce1RayCount\": %u, \"probedInstid\": %d, "
		"\"probedTriid\": %d, \"traceTime0\": %g, \"traceTime1\": %g, \"SMcount\": %u}\n",
		calls, frames, st.primaryRayCount, st.bounce1RayCount, st.probedInstid, st.probedTriid, st.traceTime0, st.traceTime1, st.SMcount );
	if (getAccumulator && w && h)
	{
		std::vector<float> acc( (size_t)w * h * 4 );
		if (getAccumulator( core, acc.data() ) != 0) return fail( "lh2_core_get_accumulator failed" );
		FILE* o = std::fopen( argv[3], "wb" );
		if (!o) return fail( "cannot write accumulator" );
		std::fwrite( acc.data(), sizeof( float ), acc.size(), o );
		std::fclose( o );
	}
	core->Shutdown();
	destroy();
	dlclose( lib );
	return 0;
}
