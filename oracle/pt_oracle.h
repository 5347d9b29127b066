/* pt_oracle.h - CPU restatement of the RenderCore_OptixPrime_B hot path (TEST INFRASTRUCTURE).

   This library is the parity CHECKER for lighthouse2_amd (the MI355X render core).  Only
   tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is never
   linked into, called by, or shipped with the product library.

   Parity status: traversal arithmetic of the parity target lives in the closed OptiX Prime
   6.0 binary, so hit decisions are defined by this restatement (Möller–Trumbore,
   open interval (tmin,tmax), tie rule (t, instance, triangle) lexicographic) and PINNED against
   the compiled reference CPU traversal RenderCore_Bart (oracle/_ref, tests/test_oracle_ref.py)
   plus committed golden vectors in tests/golden/.  Shading follows the reference kernels
   line by line; see the per-function citations in pt_oracle.c.
*/
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include "../include/lh2_core_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct Oracle Oracle;

typedef struct
{
	uint32_t rayCount[16];      /* extension rays traced per path length 1..16 */
	uint32_t shadowRays;        /* shadow rays generated (all bounces)         */
	uint32_t maxPathLength;     /* deepest bounce executed                      */
	int probedInstid, probedTriid; float probedDist;
} OracleStats;

Oracle* orc_create( void );
void orc_destroy( Oracle* o );
void orc_set_bluenoise( Oracle* o, const uint8_t* table327680 );
void orc_set_max_path_length( Oracle* o, int maxPathLength );
void orc_set_geometry( Oracle* o, int meshIdx, const lh2_CoreTri* tris, int triCount );
void orc_set_geometry_many( Oracle* o, int first, int count, const lh2_CoreTri* const* tris, const int* counts, int nthreads );
void orc_set_instance( Oracle* o, int instIdx, int meshIdx, const float* mat16 );
void orc_update_toplevel( Oracle* o );
void orc_set_materials( Oracle* o, const lh2_CoreMaterial* mats, int count );
void orc_set_lights( Oracle* o, const lh2_CoreLightTri* area, int nArea, const lh2_CorePointLight* point, int nPoint,
	const lh2_CoreSpotLight* spot, int nSpot, const lh2_CoreDirectionalLight* dir, int nDir );
void orc_set_sky( Oracle* o, const float* rgb, int w, int h );
void orc_set_textures( Oracle* o, const lh2_CoreTexDesc* tex, int count );   /* before orc_set_materials */
/* one texel fetch (sampling_shared.h FetchTexel / FetchTexelTrilinear); storage 0 = ARGB32, 2 = NRM32 */
int orc_fetch_texel( const Oracle* o, int storage, float u, float v, int offset, int w, int h, float lambda, int trilinear, float* out4 );
void orc_setting( Oracle* o, const char* name, float value );
void orc_set_target( Oracle* o, int w, int h, int spp );
void orc_set_probe( Oracle* o, int x, int y );
void orc_debug_pixel( Oracle* o, int px, int cap );       /* diagnostics: log pixel px's path vertices and shadow rays */
int orc_debug_log( const Oracle* o, float* out, int cap );  /* 16 floats per record; returns the records written */
void orc_set_tile( Oracle* o, int y0, int y1 );   /* render rows [y0, y1) only (-1 = all) */
void orc_set_tile_bands( Oracle* o, int rank, int nranks, int band );   /* rows in bands, round-robin */
void orc_render( Oracle* o, const lh2_ViewPyramid* view, int converge, int nthreads );
void orc_get_accumulator( const Oracle* o, float* out4 );     /* w*h float4, raw */
int  orc_samples_taken( const Oracle* o );
void orc_get_stats( const Oracle* o, OracleStats* s );

/* unit-level entry points (used by the kernel-level parity tests) */
void orc_generate_eye_rays( Oracle* o, const lh2_ViewPyramid* view, uint32_t R0, int pass,
	float* orgTmin4, float* dirTmax4, float* state8 );
/* closest hit: hits4 = {t, triid, instid, uv16} as 4 x 32-bit (t<0 / triid=-1 on miss);
   visits2 (optional) = {node records read (32 B each), triangles tested} per ray */
void orc_trace_closest( const Oracle* o, const float* orgTmin4, const float* dirTmax4, int n,
	uint32_t* hits4, uint32_t* visits2, int nthreads );
/* any hit: bit i of occluded[i>>5] set when ray i hits anything in (tmin, tmax) */
void orc_trace_any( const Oracle* o, const float* orgTmin4, const float* dirTmax4, int n, uint32_t* occluded );

/* lights (lights_shared.h:36-261) on the lights of orc_set_lights: light i's potential (area, point, spot, directional
   order; bary / areaI as RandomPointOnLight / LightPickProb pass them), LightPickProb, RandomBarycentrics, and
   RandomPointOnLight (out8: point xyz, pickProb, lightPdf, lightColor rgb) */
float orc_light_potential( const Oracle* o, int i, const float* I3, const float* N3, const float* bary3, const float* areaI3 );
float orc_light_pick_prob( const Oracle* o, int idx, const float* O3, const float* N3, const float* I3 );
void orc_random_barycentrics( float r0, float* out3 );
void orc_random_point_on_light( const Oracle* o, float r0, float r1, const float* I3, const float* N3, float* out8 );

/* numerics KATs */
uint32_t orc_wanghash( uint32_t s );
uint32_t orc_xorshift( uint32_t s );
float orc_bluenoise( const Oracle* o, int x, int y, int sampleIndex, int dim );
uint32_t orc_pack_normal( float x, float y, float z );
void orc_unpack_normal( uint32_t p, float* out3 );
void orc_mat4_inverse( const float* m16, float* out16 );
void orc_detmath_eval( int fn, const float* x, const float* y, int n, float* out );

#ifdef __cplusplus
}
#endif

#endif
