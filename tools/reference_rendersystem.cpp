/* reference_rendersystem.cpp - replay a recorded call stream through libRenderCore_MI355X.so using the
   REFERENCE's own interface declaration: the only header of the boundary is
   /root/reference/lib/RenderSystem/core_api_base.h (with platform.h, as every RenderSystem TU includes
   it), compiled with the layout probe's typedef shims (tests/test_abi_layout.py REF_FLAGS; nothing of
   this repository's include/ is used).  So every call site below is the reference's: argument types
   and passing conventions come from its CoreAPI_Base, e.g.
     CoreStats GetCoreStats()                       returned by value (sret pointer)  core_api_base.h:84
     SetProbePos( const int2 pos )                  int2 by value                     core_api_base.h:88
     SetTarget( GLTexture* target, const uint spp ) the reference GLTexture class       core_api_base.h:90
     Render( const ViewPyramid& view, const Convergence converge )   enum by value      core_api_base.h:94
     SetSkyData( ..., const mat4& worldToLight )    SetInstance( ..., const mat4& )     core_api_base.h:107,111
   The core is loaded as RenderSystem loads it (core_api_base.cpp:97-132: dlopen RTLD_NOW | RTLD_GLOBAL,
   dlsym CreateCore / DestroyCore, Init() again).  GLTexture's constructors live in the reference's
   platform library (they create a GL texture), so the target is a GLTexture-typed view of its three
   data members (ID 0: headless), the one thing the core reads.

   The call stream comes from lighthouse2_amd/record.py (CallRecorder); the accumulator is read back with
   the core's headless extension lh2_core_get_accumulator (resolved with dlsym, no header).

   Build (oracle/Makefile.ref, only where /root/reference exists; the binary travels to the GPU box):
     g++ -O2 -std=c++17 <REF_FLAGS> tools/reference_rendersystem.cpp -ldl -o oracle/_ref/reference_rendersystem
   Run: reference_rendersystem <lib.so> <calls.bin> <accumulator.out> [--parse-only]
*/
#include "platform.h"
#include "core_api_base.h"

#include <dlfcn.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

using namespace lighthouse2;

namespace {

enum Op : uint32_t { SET_SKY = 1, SET_MATERIALS, SET_GEOMETRY, SET_INSTANCE, UPDATE_TOPLEVEL, SET_LIGHTS, SETTING, SET_TARGET, RENDER, SET_PROBE, SET_TEXTURES };

struct Reader
{
	const uint8_t* p; size_t n, off = 0;
	template <class T> T get() { T v; std::memcpy( &v, p + off, sizeof( T ) ); off += sizeof( T ); return v; }
	const uint8_t* take( size_t bytes ) { const uint8_t* q = p + off; off += bytes; return q; }
};

/* the recorded bytes are the reference structs' bytes (record.py packs lighthouse2_amd/abi.py types, whose
   layouts tests/test_abi_layout.py checks against these same headers) */
template <class T> std::vector<T> copy_array( Reader& r, size_t count )
{
	std::vector<T> v( count ? count : 1 );
	if (count) std::memcpy( (void*)v.data(), r.take( sizeof( T ) * count ), sizeof( T ) * count );
	return v;
}

int fail( const char* msg ) { std::fprintf( stderr, "reference_rendersystem: %s\n", msg ); return 1; }

/* GLTexture's data members (system.h:251-252) without its GL-creating constructor */
struct GLTextureData { GLuint ID; uint width, height; };
static_assert( sizeof( GLTextureData ) == sizeof( GLTexture ), "GLTexture layout" );

}  // namespace

int main( int argc, char** argv )
{
	if (argc < 4) return fail( "usage: reference_rendersystem <lib.so> <calls.bin> <accumulator.out> [--parse-only]" );
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
		lib = dlopen( argv[1], RTLD_NOW | RTLD_GLOBAL );                 /* core_api_base.cpp:97-110 */
		if (!lib) return fail( dlerror() );
		auto create = (CoreAPI_Base * (*)()) dlsym( lib, "CreateCore" );   /* core_api_base.cpp:124-127 */
		destroy = (void (*)()) dlsym( lib, "DestroyCore" );
		getAccumulator = (int (*)( void*, float* )) dlsym( lib, "lh2_core_get_accumulator" );
		if (!create || !destroy) return fail( "CreateCore/DestroyCore not exported" );
		core = create();
		core->Init();                                                         /* core_api_base.cpp:129 */
	}

	alignas( GLTexture ) unsigned char texStore[sizeof( GLTexture )];
	GLTextureData* texData = new (texStore) GLTextureData{ 0, 0, 0 };
	GLTexture* target = reinterpret_cast<GLTexture*>( texStore );
	Reader r{ buf.data(), buf.size() };
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
			texData->width = r.get<uint32_t>(), texData->height = r.get<uint32_t>();
			const uint spp = r.get<uint32_t>();
			if (core) core->SetTarget( target, spp );
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
			const int x = r.get<int>(), y = r.get<int>();
			if (core) core->SetProbePos( make_int2( x, y ) );
			break;
		}
		case SET_TEXTURES:
		{
			/* per texture: width, height, flags, pixelCount, MIPlevels, storage, texel bytes, texels (record.py); the
			   descriptors point at this host's copies for the duration of the call (rendercore.cpp:276-347) */
			const int n = r.get<int>();
			std::vector<CoreTexDesc> d( n > 0 ? n : 1 );
			std::vector<std::vector<uint8_t>> texels( n > 0 ? n : 1 );
			for (int i = 0; i < n; i++)
			{
				d[i].width = r.get<uint32_t>(), d[i].height = r.get<uint32_t>(), d[i].flags = r.get<uint32_t>();
				d[i].pixelCount = r.get<uint32_t>(), d[i].MIPlevels = r.get<uint32_t>();
				d[i].storage = (TexelStorage)r.get<int32_t>();
				d[i].firstPixel = 0;
				const uint32_t bytes = r.get<uint32_t>();
				const uint8_t* src = r.take( bytes );
				texels[i].assign( src, src + bytes );
				d[i].idata = (uchar4*)(void*)texels[i].data();
			}
			if (core) core->SetTextures( d.data(), n );
			break;
		}
		case SET_MATERIALS:
		{
			const int n = r.get<int>();
			auto m = copy_array<CoreMaterial>( r, n );
			if (core) core->SetMaterials( m.data(), n );
			break;
		}
		case SET_LIGHTS:
		{
			const int na = r.get<int>(), np = r.get<int>(), ns = r.get<int>(), nd = r.get<int>();
			auto a = copy_array<CoreLightTri>( r, na );
			auto p = copy_array<CorePointLight>( r, np );
			auto s = copy_array<CoreSpotLight>( r, ns );
			auto d = copy_array<CoreDirectionalLight>( r, nd );
			if (core) core->SetLights( a.data(), na, p.data(), np, s.data(), ns, d.data(), nd );
			break;
		}
		case SET_SKY:
		{
			const uint32_t sw = r.get<uint32_t>(), sh = r.get<uint32_t>();
			auto px = copy_array<float3>( r, (size_t)sw * sh );
			if (core) core->SetSkyData( px.data(), sw, sh, mat4::Identity() );
			break;
		}
		case SET_GEOMETRY:
		{
			const int idx = r.get<int>(), n = r.get<int>();
			auto verts = copy_array<float4>( r, (size_t)3 * n );
			auto tris = copy_array<CoreTri>( r, n );
			if (core) core->SetGeometry( idx, verts.data(), 3 * n, n, tris.data(), nullptr );
			break;
		}
		case SET_INSTANCE:
		{
			const int idx = r.get<int>(), mesh = r.get<int>();
			mat4 T;
			std::memcpy( (void*)&T, r.take( 64 ), 64 );
			if (core) core->SetInstance( idx, mesh, T );
			break;
		}
		case UPDATE_TOPLEVEL:
			if (core) core->UpdateToplevel();
			break;
		case RENDER:
		{
			ViewPyramid view;
			std::memcpy( (void*)&view, r.take( sizeof( view ) ), sizeof( view ) );
			const int converge = r.get<int>();
			if (core) core->Render( view, converge ? Restart : Converge );
			frames++;
			break;
		}
		default: return fail( "unknown opcode" );
		}
		if (r.off != end) return fail( "payload size mismatch" );
	}
	if (parseOnly)
	{
		std::printf( "{\"calls\": %d, \"frames\": %d, \"width\": %u, \"height\": %u}\n", calls, frames, texData->width, texData->height );
		return 0;
	}
	const CoreStats st = core->GetCoreStats();   /* by value through the reference vtable */
	std::printf( "{\"calls\": %d, \"frames\": %d, \"primaryRayCount\": %u, \"bounce1RayCount\": %u, \"probedInstid\": %d, "
		"\"probedTriid\": %d, \"traceTime0\": %g, \"traceTime1\": %g, \"SMcount\": %u, \"deviceName\": \"%s\"}\n",
		calls, frames, st.primaryRayCount, st.bounce1RayCount, st.probedInstid, st.probedTriid, st.traceTime0, st.traceTime1, st.SMcount,
		st.deviceName ? st.deviceName : "" );
	const uint32_t w = texData->width, h = texData->height;
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
