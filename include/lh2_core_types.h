/* lh2_core_types.h - ABI-compatible POD re-declarations of the Lighthouse 2 RenderCore types.

   These are NOT copies of the reference headers; they are independent declarations whose
   size / offset / alignment must equal the reference's x86-64 (g++/clang, Itanium ABI) layout.
   tests/test_abi_layout.py compiles a probe against /root/reference/lib/RenderSystem headers (when
   present) and checks every size and offset listed here; the Python ctypes mirror in
   lighthouse2_amd/abi.py is checked against the same numbers.

   Reference declarations (file:line, relative to /root/reference/lib):
     int2/float2 ALIGN(8), float4/int4/uint4 ALIGN(16)          RenderSystem/common_types.h:58-78
     mat4 { float cell[16] } (row-major)                         RenderSystem/common_types.h:469-473
     Convergence                                                 RenderSystem/common_classes.h:38-42
     CoreTri (176 B)                                             RenderSystem/common_classes.h:57-91
     CoreTri4 (176 B, quad-float view)                           RenderSystem/common_classes.h:126-154
     CoreInstanceDesc (80 B)                                     RenderSystem/common_classes.h:163-170
     CoreMaterial (688 B) + Vec3Value (40) + ScalarValue (32)    RenderSystem/common_classes.h:177-238
     CoreTexDesc (40 B, host view)                               RenderSystem/common_classes.h:246-269
     CoreLightTri 96 / CorePointLight 32 / CoreSpotLight 48 /
     CoreDirectionalLight 32                                     RenderSystem/common_classes.h:275-356
     ViewPyramid (68 B)                                          RenderSystem/common_classes.h:362-385
     CoreStats (104 B)                                           RenderSystem/core_api_base.h:30-61
     GLTexture data members { GLuint ID; uint width, height; }   platform/system.h:233-253
*/
#ifndef LH2_CORE_TYPES_H
#define LH2_CORE_TYPES_H

#ifdef __cplusplus
#include <cstdint>
#include <cstddef>
#define LH2_ALIGN(x) alignas(x)
#else
#include <stdint.h>
#include <stddef.h>
#define LH2_ALIGN(x) _Alignas(x)
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } lh2_float3;
typedef struct { LH2_ALIGN(8) float x; float y; } lh2_float2;
typedef struct { LH2_ALIGN(8) int x; int y; } lh2_int2;
typedef struct { LH2_ALIGN(16) float x; float y, z, w; } lh2_float4;
typedef struct { LH2_ALIGN(16) uint32_t x; uint32_t y, z, w; } lh2_uint4;
typedef struct { float cell[16]; } lh2_mat4;

enum { LH2_CONVERGE = 0, LH2_RESTART = 1 };

/* CoreTri: host-side triangle record, 176 bytes. */
typedef struct
{
	float u0, u1, u2;      int ltriIdx;   /*   0 */
	float v0, v1, v2;      uint32_t material; /* 16 */
	lh2_float3 vN0;        float Nx;      /*  32 */
	lh2_float3 vN1;        float Ny;      /*  48 */
	lh2_float3 vN2;        float Nz;      /*  64 */
	lh2_float3 T;          float area;    /*  80 */
	lh2_float3 B;          float invArea; /*  96 */
	lh2_float3 alpha;      float LOD;     /* 112 */
	lh2_float3 vertex0;    float dummy0;  /* 128 */
	lh2_float3 vertex1;    float dummy1;  /* 144 */
	lh2_float3 vertex2;    float dummy2;  /* 160 */
} lh2_CoreTri;

typedef struct
{
	lh2_float3 value; int textureID; float scale; lh2_float2 uvscale, uvoffset;
} lh2_Vec3Value;                 /* 40 B */
typedef struct
{
	float value; int textureID; int component; float scale; lh2_float2 uvscale, uvoffset;
} lh2_ScalarValue;               /* 32 B */

typedef struct
{
	lh2_Vec3Value color, detailColor, normals, detailNormals;   /*   0 .. 160 */
	uint32_t flags;                                              /* 160 */
	lh2_Vec3Value absorption;                                    /* 168 */
	lh2_ScalarValue metallic, subsurface, specular, roughness,   /* 208 .. */
		specularTint, anisotropic, sheen, sheenTint, clearcoat, clearcoatGloss, transmission, eta;
	lh2_ScalarValue reflection, refraction, ior;                 /* 592 .. 688 */
} lh2_CoreMaterial;

typedef struct
{
	void* idata;            /* union { float4* fdata; uchar4* idata; } */
	uint32_t width, height, flags, pixelCount, firstPixel, MIPlevels;
	int32_t storage;        /* TexelStorage: ARGB32=0, ARGB128, NRM32 */
} lh2_CoreTexDesc;          /* 40 B */

typedef struct
{
	lh2_float3 centre; float energy;
	lh2_float3 N; float area;
	lh2_float3 radiance; int dummy2;
	lh2_float3 vertex0; int triIdx;
	lh2_float3 vertex1; int instIdx;
	lh2_float3 vertex2; int dummy1;
} lh2_CoreLightTri;         /* 96 B */
typedef struct { lh2_float3 position; float energy; lh2_float3 radiance; int dummy; } lh2_CorePointLight;
typedef struct { lh2_float3 position; float cosInner; lh2_float3 radiance; float cosOuter; lh2_float3 direction; int dummy; } lh2_CoreSpotLight;
typedef struct { lh2_float3 direction; float energy; lh2_float3 radiance; int dummy; } lh2_CoreDirectionalLight;

typedef struct
{
	lh2_float3 pos, p1, p2, p3;
	float aperture, spreadAngle, imagePlane, focalDistance, distortion;
} lh2_ViewPyramid;          /* 68 B */

typedef struct
{
	char* deviceName;
	uint32_t SMcount, ccMajor, ccMinor, VRAM;
	uint32_t argb32TexelCount, argb128TexelCount, nrm32TexelCount;
	float bvhBuildTime;
	uint32_t totalRays, totalExtensionRays, totalShadowRays;
	float renderTime;
	uint32_t primaryRayCount; float traceTime0;
	uint32_t bounce1RayCount; float traceTime1;
	uint32_t deepRayCount;    float traceTimeX;
	float shadowTraceTime, shadeTime, filterTime;
	int probedInstid, probedTriid; float probedDist;
} lh2_CoreStats;            /* 104 B */

/* Data members of lighthouse2::GLTexture (no virtuals): what SetTarget reads. ID == 0 = headless. */
typedef struct { uint32_t ID; uint32_t width, height; } lh2_GLTexture;

/* Device-side instance descriptor used by shading (same layout as CoreInstanceDesc). */
typedef struct
{
	void* triangles;                 /* device pointer to CoreTri4[] of the mesh */
	int dummy1, dummy2;
	lh2_float4 A, B, C, D;           /* rows of the inverse transform */
} lh2_CoreInstanceDesc;              /* 80 B */

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* LH2_CORE_TYPES_H */
