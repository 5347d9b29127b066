/* lh2_rendercore.h - flat C-ABI of libRenderCore_MI355X.so.

   Two layers, both exported with default visibility:

   1. The reference boundary, unchanged:  CoreAPI_Base* CreateCore(); void DestroyCore();
      (RenderCore_OptixPrime_B/core_api.h:63-64, core_api.cpp:20-34; declared in lh2_core_api.hpp).

   2. A flat extern "C" mirror of the same 14 CoreAPI_Base methods, for hosts that cannot call a
      C++ vtable (ctypes / cgo / JNI / N-API).  Every lh2_core_* call below goes THROUGH the
      CoreAPI_Base vtable of the object it is given, exactly as RenderSystem does
      (rendersystem.cpp:22-301), so the flat layer exercises the same entry points.  Each returns
      0 on success and -1 on a fatal error (message in lh2_last_error()), instead of the
      reference's FatalError -> exit(0) (platform/system.cpp:221-236), which the vtable path keeps.

   Reference interface each entry replaces (file:line under /root/reference/lib):
     lh2_core_new / lh2_core_delete      CreateCore / DestroyCore       RenderCore_OptixPrime_B/core_api.cpp:20-34
     lh2_core_init                       CoreAPI_Base::Init             RenderSystem/core_api_base.h:86
     lh2_core_get_stats                  CoreAPI_Base::GetCoreStats     core_api_base.h:84
     lh2_core_set_probe                  CoreAPI_Base::SetProbePos      core_api_base.h:88
     lh2_core_set_target                 CoreAPI_Base::SetTarget        core_api_base.h:90
     lh2_core_setting                    CoreAPI_Base::Setting          core_api_base.h:92
     lh2_core_render                     CoreAPI_Base::Render           core_api_base.h:94
     lh2_core_shutdown                   CoreAPI_Base::Shutdown         core_api_base.h:96
     lh2_core_set_textures               CoreAPI_Base::SetTextures      core_api_base.h:98
     lh2_core_set_materials              CoreAPI_Base::SetMaterials     core_api_base.h:100
     lh2_core_set_lights                 CoreAPI_Base::SetLights        core_api_base.h:102-105
     lh2_core_set_sky                    CoreAPI_Base::SetSkyData       core_api_base.h:107
     lh2_core_set_geometry               CoreAPI_Base::SetGeometry      core_api_base.h:109
     lh2_core_set_instance               CoreAPI_Base::SetInstance      core_api_base.h:111
     lh2_core_update_toplevel            CoreAPI_Base::UpdateToplevel   core_api_base.h:113
   Extensions (no reference counterpart; used by the tile partition, the bench and the tests):
     lh2_core_set_tile, lh2_core_set_tile_bands, lh2_core_sync, lh2_core_get_accumulator, lh2_core_get_frame,
     lh2_core_copy_accumulator_rows, lh2_core_copy_frame_async, lh2_core_pack_tile, lh2_core_pack_tile_ordered, lh2_core_tile_rows, lh2_core_stream, lh2_core_ray_counts, lh2_core_trace_closest,
     lh2_core_trace_any, lh2_core_trace_closest_device, lh2_core_generate_eye_rays,
     lh2_core_scene_info, lh2_core_debug_shadow_rays, lh2_core_debug_bvh4, lh2_core_debug_poison_tlas, lh2_core_get_setting, lh2_set_device, lh2_xorshift_floats, lh2_version.
*/
#ifndef LH2_RENDERCORE_H
#define LH2_RENDERCORE_H

#include "lh2_core_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void* lh2_core;   /* a lighthouse2::CoreAPI_Base* */

const char* lh2_version( void );
const char* lh2_last_error( void );
int lh2_set_device( int device );

int lh2_core_new( lh2_core* out );           /* like CreateCore(), but not the process singleton */
int lh2_core_delete( lh2_core core );

int lh2_core_init( lh2_core core );
int lh2_core_get_stats( lh2_core core, lh2_CoreStats* out );
int lh2_core_set_probe( lh2_core core, int x, int y );
int lh2_core_set_target( lh2_core core, uint32_t width, uint32_t height, uint32_t spp );
int lh2_core_setting( lh2_core core, const char* name, float value );
int lh2_core_get_setting( lh2_core core, const char* name, float* value );   /* extension: current value (-1: unknown name) */
int lh2_core_render( lh2_core core, const lh2_ViewPyramid* view, int converge );
int lh2_core_shutdown( lh2_core core );
int lh2_core_set_textures( lh2_core core, const lh2_CoreTexDesc* tex, int count );
int lh2_core_set_materials( lh2_core core, lh2_CoreMaterial* mats, int count );
int lh2_core_set_lights( lh2_core core, const lh2_CoreLightTri* area, int nArea, const lh2_CorePointLight* point, int nPoint,
	const lh2_CoreSpotLight* spot, int nSpot, const lh2_CoreDirectionalLight* dir, int nDir );
int lh2_core_set_sky( lh2_core core, const float* rgb, uint32_t width, uint32_t height );
int lh2_core_set_geometry( lh2_core core, int meshIdx, const float* vertexData4, int vertexCount, int triangleCount,
	const lh2_CoreTri* triangles, const uint32_t* alphaFlags );
int lh2_core_set_instance( lh2_core core, int instanceIdx, int meshIdx, const float* matrix16 );
int lh2_core_update_toplevel( lh2_core core );

int lh2_core_set_tile( lh2_core core, int y0, int y1 );                 /* render frame rows [y0, y1) (-1: to the end) */
int lh2_core_set_tile_bands( lh2_core core, int rank, int nranks, int band ); /* rows in bands of `band`, round-robin over ranks */
int lh2_core_sync( lh2_core core );
int lh2_core_get_accumulator( lh2_core core, float* out4 );
int lh2_core_get_frame( lh2_core core, float* out4 );
int lh2_core_copy_accumulator_rows( lh2_core core, void* deviceDst, int y0, int y1 );
/* the last finalized frame (w x h float4) -> deviceDst, async on the core stream: the headless display copy
   (interoptexture.cpp:51-71 copies it into the app's GL texture every frame) */
int lh2_core_copy_frame_async( lh2_core core, void* deviceDst );
int lh2_core_pack_tile( lh2_core core, void* deviceDst );   /* owned accumulator rows -> deviceDst (rows x width float4), async on the core stream */
/* the same, ordered both ways with consumerStream (a hipStream_t that reads deviceDst, e.g. the one
   the gather runs on; null: the null stream): the pack waits for the consumer's earlier work, the
   consumer for the pack */
int lh2_core_pack_tile_ordered( lh2_core core, void* deviceDst, void* consumerStream );
int lh2_core_tile_rows( lh2_core core, int* rows );
int lh2_core_stream( lh2_core core, void** hipStream );     /* the core's HIP stream (order other streams after its work) */
int lh2_core_ray_counts( lh2_core core, uint32_t* out17 );
int lh2_core_trace_closest( lh2_core core, const float* orgTmin4, const float* dirTmax4, int n, uint32_t* hits4 );
int lh2_core_trace_any( lh2_core core, const float* orgTmin4, const float* dirTmax4, int n, uint32_t* occluded );
int lh2_core_trace_closest_device( lh2_core core, const void* rayO, const void* rayD, int n, void* hits, int iterations, float* msPerLaunch );
int lh2_core_generate_eye_rays( lh2_core core, const lh2_ViewPyramid* view, uint32_t R0, int pass, float* orgTmin4, float* dirTmax4, float* state8 );
int lh2_core_scene_info( lh2_core core, int* nodeCount, int* triCount, int* maxDepth, int* instCount );
/* diagnostics: the last frame's queued shadow rays (at most cap): {O, tmin}, {D, tmax}, {potential rgb, pixel index bits} */
int lh2_core_debug_shadow_rays( lh2_core core, float* o4, float* d4, float* p4, int cap, int* n );
/* diagnostics: the scene's BVH4 nodes (BLAS then TLAS, at most cap): f32 (32 floats each) and quantized (16 words
   each, the layout of k_quantize4); *n = the nodes copied */
/* cap 0 (or null arrays): *n = the node count, nothing copied */
int lh2_core_debug_bvh4( lh2_core core, float* f32Nodes, uint32_t* qNodes, int cap, int* n );
/* test hook: fill both TLAS slots' node regions with `value` (stale memory behind the nodes a TLAS update writes) */
int lh2_core_debug_poison_tlas( lh2_core core, float value );

/* host utility: n successive RandomFloat() values of Marsaglia xorshift32 (platform/system.cpp:44-46) */
int lh2_xorshift_floats( uint32_t seed, float* out, uint64_t n );

#ifdef __cplusplus
}
#endif

#endif
