/* lh2_core_api.hpp - ABI-compatible declaration of lighthouse2::CoreAPI_Base (C++ only).

   The drop-in boundary of a Lighthouse 2 render core is a C++ object returned by the exported
   C symbol CreateCore(); RenderSystem calls it through this vtable
   (RenderSystem/core_api_base.h:78-114; loader core_api_base.cpp:97-132).  This declaration
   keeps the reference's virtual-function ORDER and parameter types (Itanium C++ ABI, g++/clang
   on Linux), using the POD mirrors of include/lh2_core_types.h, so that an unchanged
   RenderSystem can load libRenderCore_MI355X.so.  There is no virtual destructor (as in the
   reference).  tests/test_abi_layout.py checks the slot order against the reference header
   (when /root/reference is present), and tools/headless_rendersystem.cpp drives a core through
   this vtable the way RenderSystem does (tests/test_boundary_replay.py).
*/
#pragma once
#include "lh2_core_types.h"

namespace lh2abi {

/* GLTexture is a class with methods but no virtuals; the core only reads its data members */
struct GLTextureView { uint32_t ID; uint32_t width, height; };

class CoreAPI_Base
{
public:
	virtual lh2_CoreStats GetCoreStats() = 0;                                             /* slot 0 */
	virtual void Init() = 0;                                                               /* 1 */
	virtual void SetProbePos( const lh2_int2 pos ) = 0;                                    /* 2 */
	virtual void SetTarget( GLTextureView* target, const uint32_t spp ) = 0;               /* 3 */
	virtual void Setting( const char* name, float value ) = 0;                             /* 4 */
	virtual void Render( const lh2_ViewPyramid& view, const int converge ) = 0;            /* 5 (Convergence enum) */
	virtual void Shutdown() = 0;                                                           /* 6 */
	virtual void SetTextures( const lh2_CoreTexDesc* tex, const int textureCount ) = 0;    /* 7 */
	virtual void SetMaterials( lh2_CoreMaterial* mat, const int materialCount ) = 0;       /* 8 */
	virtual void SetLights( const lh2_CoreLightTri* areaLights, const int areaLightCount,  /* 9 */
		const lh2_CorePointLight* pointLights, const int pointLightCount,
		const lh2_CoreSpotLight* spotLights, const int spotLightCount,
		const lh2_CoreDirectionalLight* directionalLights, const int directionalLightCount ) = 0;
	virtual void SetSkyData( const lh2_float3* pixels, const uint32_t width, const uint32_t height, const lh2_mat4& worldToLight ) = 0;  /* 10 */
	virtual void SetGeometry( const int meshIdx, const lh2_float4* vertexData, const int vertexCount, const int triangleCount,      /* 11 */
		const lh2_CoreTri* triangles, const uint32_t* alphaFlags ) = 0;
	virtual void SetInstance( const int instanceIdx, const int modelIdx, const lh2_mat4& transform ) = 0;                            /* 12 */
	virtual void UpdateToplevel() = 0;                                                                                               /* 13 */
};

}  // namespace lh2abi

/* The two symbols the reference loader resolves with dlsym (core_api_base.cpp:124-127). */
extern "C" lh2abi::CoreAPI_Base* CreateCore();
extern "C" void DestroyCore();
