/* pt_oracle.c - CPU restatement of the RenderCore_OptixPrime_B wavefront path tracer.

   TEST INFRASTRUCTURE ONLY (see pt_oracle.h).  Build: oracle/Makefile (gcc -O2 -ffp-contract=off).

   Every function cites the reference (paths relative to /root/reference/lib) it restates.
   Expressions keep the reference's evaluation order (C/C++ left-to-right, no contraction) so
   that the HIP core, which follows the same order, is bit-comparable.  Transcendentals come
   from include/lh2_detmath.h (the parity numerics contract).

   Where the reference has undefined behaviour the restatement pins one definition, and the
   HIP core implements the same one (DESIGN.md "Reference quirks"):
     Q1 SampleBSDF outputs (wiw, component pdf, contrib) start at 0 instead of uninitialised.
     Q2 point-light NEE colour: the reference shadows the out-param (lights_shared.h:228);
        we return the light's radiance.
     Q3 LightPickProb with ltriIdx outside [0, areaLightCount) returns 0.
     Q4 float->uint conversions saturate (GPU semantics), see lh2_f2u.
     Q6 blue-noise rank lookups past the end of the table read zero padding.
     Q5 light potentials are recomputed instead of stored in a MAXISLIGHTS=8 array, which the
        reference overruns for > 8 lights; values are identical for <= 8 lights.
*/
#include "pt_oracle.h"
#include "../include/lh2_detmath.h"
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <pthread.h>

#define MAXPATHLENGTH_DEFAULT 16
#define NOHIT -1
#define S_SPECULAR 1
#define S_BOUNCED 2
#define S_VIASPECULAR 4
#define S_BOUNCEDTWICE 8
#define ENOUGH_BOUNCES S_BOUNCED
#define EPSILON 0.0001f
#define INVPI LH2_INVPI
#define PI LH2_PI
#define TWOPI LH2_TWOPI

/* ------------------------------------------------------------------------------------- */
/* vector helpers: helper_math.h semantics (CUDA/helper_math.h), explicit evaluation order  */
/* ------------------------------------------------------------------------------------- */
typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;
typedef struct { float x, y; } f2;
static inline f3 mk3( float x, float y, float z ) { f3 r = { x, y, z }; return r; }
static inline f3 s3( float s ) { return mk3( s, s, s ); }
static inline f3 add3( f3 a, f3 b ) { return mk3( a.x + b.x, a.y + b.y, a.z + b.z ); }
static inline f3 sub3( f3 a, f3 b ) { return mk3( a.x - b.x, a.y - b.y, a.z - b.z ); }
static inline f3 mul3( f3 a, f3 b ) { return mk3( a.x * b.x, a.y * b.y, a.z * b.z ); }
static inline f3 muls( f3 a, float s ) { return mk3( a.x * s, a.y * s, a.z * s ); }
static inline f3 smul( float s, f3 a ) { return mk3( s * a.x, s * a.y, s * a.z ); }
static inline f3 divs( f3 a, float s ) { return mk3( a.x / s, a.y / s, a.z / s ); }
static inline f3 adds( f3 a, float s ) { return mk3( a.x + s, a.y + s, a.z + s ); }
static inline f3 sadd( float s, f3 a ) { return mk3( s + a.x, s + a.y, s + a.z ); }
static inline f3 neg3( f3 a ) { return mk3( -a.x, -a.y, -a.z ); }
static inline float dot3( f3 a, f3 b ) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline f3 cross3( f3 a, f3 b ) { return mk3( a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x ); }
static inline float length3( f3 v ) { return sqrtf( dot3( v, v ) ); }
/* normalize = v * rsqrtf(dot(v,v)), host rsqrtf = 1/sqrtf (helper_math.h:62,1309) */
static inline f3 normalize3( f3 v ) { const float invLen = 1.0f / sqrtf( dot3( v, v ) ); return muls( v, invLen ); }
static inline f3 reflect3( f3 i, f3 n ) { return sub3( i, muls( smul( 2.0f, n ), dot3( n, i ) ) ); } /* helper_math.h:1411 */
static inline float lerpf_( float a, float b, float t ) { return a + t * (b - a); }                   /* helper_math.h:1130 */
static inline float saturatef_( float x ) { return fmaxf( 0.0f, fminf( 1.0f, x ) ); }
static inline float sqrf( float x ) { return x * x; }
static inline float mixf( float a, float b, float x ) { return x <= 0 ? a : x >= 1 ? b : lerpf_( a, b, x ); } /* tools_shared.h:98 */
static inline float clampf_( float f, float a, float b ) { return fmaxf( a, fminf( f, b ) ); }
static inline f3 f4xyz( f4 a ) { return mk3( a.x, a.y, a.z ); }
static inline uint32_t fbits( float f ) { return lh2_f2b( f ); }
static inline float bitsf( uint32_t u ) { return lh2_b2f( u ); }
static inline int isfinite_( float x ) { return x == x && x - x == 0.0f; }
static inline f3 lf3( lh2_float3 a ) { return mk3( a.x, a.y, a.z ); }

/* ------------------------------------------------------------------------------------- */
/* RNG + blue noise: tools_shared.h:60-62, 336-350; platform/system.cpp:44-49              */
/* ------------------------------------------------------------------------------------- */
static inline uint32_t WangHash( uint32_t s ) { s = (s ^ 61) ^ (s >> 16), s *= 9, s = s ^ (s >> 4), s *= 0x27d4eb2d, s = s ^ (s >> 15); return s; }
static inline uint32_t RandomInt( uint32_t* s ) { *s ^= *s << 13, *s ^= *s >> 17, *s ^= *s << 5; return *s; }
static inline float RandomFloat( uint32_t* s ) { return (float)RandomInt( s ) * 2.3283064365387e-10f; }

/* ------------------------------------------------------------------------------------- */
/* scene                                                                                   */
/* ------------------------------------------------------------------------------------- */
typedef struct { f3 bmin; int first; f3 bmax; int count; } BNode; /* Bart BVHNode, bvh.h:10-15 */

typedef struct
{
	int triCount;
	lh2_CoreTri* tris;
	f3* centers; f3* tmin; f3* tmax;
	BNode* pool; int poolPtr;
	int* idx;
	f3 aabbMin, aabbMax;
} Mesh;

typedef struct { int mesh; float T[16]; float inv[16]; f3 wmin, wmax; } Instance;

typedef struct
{
	/* CUDAMaterial-equivalent (core_settings.h:94-104) after the host conversion */
	uint16_t diffuse[3], transmittance[3]; uint32_t flags;
	uint32_t params[4];
	uint32_t maps[6][4];   /* tex0, tex1, nmap0, nmap1, smap, rmap: {w | h << 16, half uvscale, half uvoffs, firstPixel} */
} Mat;

struct Oracle
{
	uint32_t* blueNoise; /* 5*65536 entries, rendercore.cpp:126-133 */
	int maxPathLength;
	Mesh* meshes; int meshCount;
	Instance* inst; int instCount, instCap;
	Mat* mats; int matCount;
	lh2_CoreLightTri* area; int nArea;
	lh2_CorePointLight* point; int nPoint;
	lh2_CoreSpotLight* spot; int nSpot;
	lh2_CoreDirectionalLight* dirl; int nDir;
	float* sky; int skyW, skyH;
	lh2_CoreTexDesc* tex; int texCount;    /* copies; firstPixel assigned per storage type */
	uint32_t* argb32; uint32_t argb32Count;
	uint32_t* nrm32; uint32_t nrm32Count;
	float spreadAngle;                    /* of the view being rendered (texture LOD cone) */
	int primeRef;                         /* RenderCore_PrimeRef validation mode */
	float geometryEpsilon, clampValue;
	int w, h, spp;
	float* acc;          /* float4 per pixel */
	int samplesTaken;
	int firstConvergingFrame;
	uint32_t camRNGseed;
	int probeX, probeY;
	int tileY0, tileY1;
	int bandRank, bandCount, band;   /* band partition (0 bands = contiguous tile) */
	OracleStats stats;
	/* diagnostics (orc_debug_pixel): every path vertex and shadow ray of one pixel, 16 floats per record */
	int debugPixel;
	float* debugLog; int debugCount, debugCap;
};
/* one debug record: kind (0 vertex: pathLength, hit t, tri, inst, ray O, D; 1 shadow ray: pathLength,
   occluded, O, D, tmax, contribution) */
static void debug_log( const Oracle* o, const float* rec )
{
	/* the debug pixel's samples and shadow rays may run on different render_worker threads (spp > 1, chunked
	   jobs): the slot is claimed with an atomic fetch-add, the count clamped when read */
	Oracle* m = (Oracle*)o;
	const int slot = __atomic_fetch_add( &m->debugCount, 1, __ATOMIC_RELAXED );
	if (slot < m->debugCap) memcpy( m->debugLog + 16 * slot, rec, 16 * sizeof( float ) );
}

Oracle* orc_create( void )
{
	Oracle* o = (Oracle*)calloc( 1, sizeof( Oracle ) );
	o->maxPathLength = MAXPATHLENGTH_DEFAULT;
	o->geometryEpsilon = 0.0f;   /* __constant__ default until Setting("epsilon") (.cuda.cu:38) */
	o->clampValue = 10.0f;       /* RenderCore::Init SetClampValue(10) (rendercore.cpp:124) */
	o->camRNGseed = 0x12345678;
	o->firstConvergingFrame = 0;
	o->tileY0 = 0, o->tileY1 = -1;
	o->debugPixel = -1;
	return o;
}

static void free_mesh( Mesh* m )
{
	free( m->tris ); free( m->centers ); free( m->tmin ); free( m->tmax ); free( m->pool ); free( m->idx );
}

void orc_destroy( Oracle* o )
{
	if (!o) return;
	for (int i = 0; i < o->meshCount; i++) free_mesh( &o->meshes[i] );
	free( o->meshes ); free( o->inst ); free( o->mats ); free( o->area ); free( o->point ); free( o->spot );
	free( o->dirl ); free( o->sky ); free( o->acc ); free( o->blueNoise );
	free( o->tex ); free( o->argb32 ); free( o->nrm32 ); free( o->debugLog );
	free( o );
}

void orc_set_bluenoise( Oracle* o, const uint8_t* t )
{
	free( o->blueNoise );
	/* Q6: blueNoiseSampler reads up to 248 entries past the 5*65536 table for sample dimensions > 7
	   near pixel (127,127) (tools_shared.h:343 vs rendercore.cpp:127); the padding is defined as 0 */
	o->blueNoise = (uint32_t*)calloc( 65536 * 5 + 256, sizeof( uint32_t ) );
	for (int i = 0; i < 65536 * 5; i++) o->blueNoise[i] = t[i];
}

void orc_set_max_path_length( Oracle* o, int m ) { o->maxPathLength = m < 1 ? 1 : m > 16 ? 16 : m; }

/* blueNoiseSampler, tools_shared.h:336-350 */
static inline float blueNoiseSampler( const uint32_t* blueNoise, int x, int y, int sampleIndex, int sampleDimension )
{
	x &= 127, y &= 127, sampleIndex &= 255, sampleDimension &= 255;
	int rankedSampleIndex = (sampleIndex ^ (int)blueNoise[sampleDimension + (x + y * 128) * 8 + 65536 * 3]) & 255;
	int value = (int)blueNoise[sampleDimension + rankedSampleIndex * 256];
	value ^= (int)blueNoise[(sampleDimension & 7) + (x + y * 128) * 8 + 65536];
	return (0.5f + (float)value) * (1.0f / 256.0f);
}

/* ------------------------------------------------------------------------------------- */
/* BVH2 build: restatement of RenderCore_Bart/bvh.cpp:57-256 (binned SAH, 8 planes/axis,    */
/* leaf if count < 4 or no split beats base cost - EPSILON).                               */
/* ------------------------------------------------------------------------------------- */
static float bart_split_cost( const Mesh* m, const int* indices, int first, int count ) /* bvh.cpp:76-94 */
{
	f3 mn = s3( FLT_MAX ), mx = s3( -FLT_MAX );
	for (int i = first; i < first + count; i++)
	{
		const f3 a = m->tmin[indices[i]], b = m->tmax[indices[i]];
		mn = mk3( fminf( mn.x, a.x ), fminf( mn.y, a.y ), fminf( mn.z, a.z ) );
		mx = mk3( fmaxf( mx.x, b.x ), fmaxf( mx.y, b.y ), fmaxf( mx.z, b.z ) );
	}
	const f3 d = sub3( mx, mn );
	const float area = 2 * d.x * d.y + 2 * d.x * d.z + 2 * d.y * d.z;
	return (float)count * area;
}
static inline float getc( f3 v, int i ) { return i == 0 ? v.x : i == 1 ? v.y : v.z; }

static int bart_partition( Mesh* m, BNode* node, int* indices, int* counts ) /* bvh.cpp:96-178 */
{
	const int bins = 8;
	int* left = (int*)malloc( sizeof( int ) * node->count );
	int* right = (int*)malloc( sizeof( int ) * node->count );
	const float base = bart_split_cost( m, m->idx, node->first, node->count );
	float best = FLT_MAX, bestPos = 0; int bestAxis = -1;
	f3 cmn = s3( FLT_MAX ), cmx = s3( -FLT_MAX );
	for (int i = node->first; i < node->first + node->count; i++)
	{
		const f3 c = m->centers[m->idx[i]];
		cmn = mk3( fminf( cmn.x, c.x ), fminf( cmn.y, c.y ), fminf( cmn.z, c.z ) );
		cmx = mk3( fmaxf( cmx.x, c.x ), fmaxf( cmx.y, c.y ), fmaxf( cmx.z, c.z ) );
	}
	for (int a = 0; a < 3; a++)
	{
		if (getc( cmn, a ) == getc( cmx, a )) continue;
		const float interval = (getc( cmx, a ) - getc( cmn, a )) / bins;
		for (int j = 0; j < bins; j++)
		{
			const float pos = getc( cmn, a ) + j * interval;
			counts[0] = counts[1] = 0;
			for (int k = node->first; k < node->first + node->count; k++)
			{
				const int t = m->idx[k];
				if (getc( m->centers[t], a ) <= pos) left[counts[0]++] = t; else right[counts[1]++] = t;
			}
			const float cost = bart_split_cost( m, left, 0, counts[0] ) + bart_split_cost( m, right, 0, counts[1] );
			if (cost + EPSILON < best) best = cost, bestAxis = a, bestPos = pos;
		}
	}
	if (base - EPSILON < best) { free( left ); free( right ); return 0; }
	counts[0] = counts[1] = 0;
	for (int i = node->first; i < node->first + node->count; i++)
	{
		const int t = m->idx[i];
		if (getc( m->centers[t], bestAxis ) <= bestPos) left[counts[0]++] = t; else right[counts[1]++] = t;
	}
	for (int i = 0; i < counts[0]; i++) indices[i] = left[i];
	for (int i = 0; i < counts[1]; i++) indices[counts[0] + i] = right[i];
	free( left ); free( right );
	return 1;
}

static void bart_subdivide( Mesh* m, int nodeIdx ) /* bvh.cpp:180-224 (iterative form) */
{
	int* stack = (int*)malloc( sizeof( int ) * (2 * m->triCount + 2) );
	int sp = 0;
	stack[sp++] = nodeIdx;
	while (sp)
	{
		BNode* node = &m->pool[stack[--sp]];
		if (node->count < 4) continue;
		int* indices = (int*)malloc( sizeof( int ) * node->count );
		int counts[2] = { 0, 0 };
		if (bart_partition( m, node, indices, counts ))
		{
			for (int i = 0; i < node->count; i++) m->idx[node->first + i] = indices[i];
			BNode* l = &m->pool[m->poolPtr], * r = &m->pool[m->poolPtr + 1];
			l->first = node->first, l->count = counts[0];
			r->first = node->first + counts[0], r->count = counts[1];
			node->count = 0, node->first = m->poolPtr;
			/* Bart recurses left then right, allocating children depth-first: emulate order */
			const int li = m->poolPtr, ri = m->poolPtr + 1;
			m->poolPtr += 2;
			stack[sp++] = ri; stack[sp++] = li;
		}
		free( indices );
	}
	free( stack );
}

static void bart_update_bounds( Mesh* m ) /* bvh.cpp:226-256 */
{
	for (int i = m->poolPtr - 1; i >= 0; i--)
	{
		BNode* n = &m->pool[i];
		if (n->count == -1) continue;
		if (n->count == 0)
		{
			const BNode* l = &m->pool[n->first], * r = &m->pool[n->first + 1];
			n->bmin = mk3( fminf( l->bmin.x, r->bmin.x ), fminf( l->bmin.y, r->bmin.y ), fminf( l->bmin.z, r->bmin.z ) );
			n->bmax = mk3( fmaxf( l->bmax.x, r->bmax.x ), fmaxf( l->bmax.y, r->bmax.y ), fmaxf( l->bmax.z, r->bmax.z ) );
			continue;
		}
		n->bmin = s3( FLT_MAX ), n->bmax = s3( -FLT_MAX );
		for (int j = n->first; j < n->first + n->count; j++)
		{
			const f3 a = m->tmin[m->idx[j]], b = m->tmax[m->idx[j]];
			n->bmin = mk3( fminf( n->bmin.x, a.x ), fminf( n->bmin.y, a.y ), fminf( n->bmin.z, a.z ) );
			n->bmax = mk3( fmaxf( n->bmax.x, b.x ), fmaxf( n->bmax.y, b.y ), fmaxf( n->bmax.z, b.z ) );
		}
	}
}

/* RenderCore_Bart/rendercore.cpp:47-79 (SetGeometry) + bvh.cpp:57-74 (Rebuild) */
void orc_set_geometry( Oracle* o, int meshIdx, const lh2_CoreTri* tris, int T )
{
	if (meshIdx >= o->meshCount)
	{
		o->meshes = (Mesh*)realloc( o->meshes, sizeof( Mesh ) * (meshIdx + 1) );
		for (int i = o->meshCount; i <= meshIdx; i++) memset( &o->meshes[i], 0, sizeof( Mesh ) );
		o->meshCount = meshIdx + 1;
	}
	Mesh* m = &o->meshes[meshIdx];
	free_mesh( m );
	memset( m, 0, sizeof( Mesh ) );
	m->triCount = T;
	m->tris = (lh2_CoreTri*)malloc( sizeof( lh2_CoreTri ) * (T ? T : 1) );
	memcpy( m->tris, tris, sizeof( lh2_CoreTri ) * T );
	m->centers = (f3*)malloc( sizeof( f3 ) * (T ? T : 1) );
	m->tmin = (f3*)malloc( sizeof( f3 ) * (T ? T : 1) );
	m->tmax = (f3*)malloc( sizeof( f3 ) * (T ? T : 1) );
	m->aabbMin = s3( FLT_MAX ), m->aabbMax = s3( -FLT_MAX );
	for (int i = 0; i < T; i++)
	{
		const f3 a = lf3( tris[i].vertex0 ), b = lf3( tris[i].vertex1 ), c = lf3( tris[i].vertex2 );
		m->centers[i] = divs( add3( add3( a, b ), c ), 3.0f );
		m->tmin[i] = mk3( fminf( fminf( a.x, b.x ), c.x ), fminf( fminf( a.y, b.y ), c.y ), fminf( fminf( a.z, b.z ), c.z ) );
		m->tmax[i] = mk3( fmaxf( fmaxf( a.x, b.x ), c.x ), fmaxf( fmaxf( a.y, b.y ), c.y ), fmaxf( fmaxf( a.z, b.z ), c.z ) );
		m->aabbMin = mk3( fminf( m->aabbMin.x, m->tmin[i].x ), fminf( m->aabbMin.y, m->tmin[i].y ), fminf( m->aabbMin.z, m->tmin[i].z ) );
		m->aabbMax = mk3( fmaxf( m->aabbMax.x, m->tmax[i].x ), fmaxf( m->aabbMax.y, m->tmax[i].y ), fmaxf( m->aabbMax.z, m->tmax[i].z ) );
	}
	m->idx = (int*)malloc( sizeof( int ) * (T ? T : 1) );
	for (int i = 0; i < T; i++) m->idx[i] = i;
	m->pool = (BNode*)malloc( sizeof( BNode ) * (2 * T + 2) );
	for (int i = 0; i < 2 * T + 2; i++) m->pool[i].count = -1, m->pool[i].first = 0;
	m->pool[0].first = 0, m->pool[0].count = T;
	m->poolPtr = 2;
	if (T > 0) { bart_subdivide( m, 0 ); bart_update_bounds( m ); }
}

/* test-infrastructure convenience: SetGeometry for meshes [first, first+count) built on nthreads threads
   (each mesh's build is the single-threaded restatement above; meshes are independent) */
typedef struct { Oracle* o; int first, count; const lh2_CoreTri* const* tris; const int* counts; int t, nt; } GeomJob;
static void* geom_worker( void* p )
{
	GeomJob* j = (GeomJob*)p;
	for (int i = j->t; i < j->count; i += j->nt) orc_set_geometry( j->o, j->first + i, j->tris[i], j->counts[i] );
	return 0;
}
void orc_set_geometry_many( Oracle* o, int first, int count, const lh2_CoreTri* const* tris, const int* counts, int nthreads )
{
	if (count <= 0) return;
	if (first + count > o->meshCount)
	{
		o->meshes = (Mesh*)realloc( o->meshes, sizeof( Mesh ) * (first + count) );
		for (int i = o->meshCount; i < first + count; i++) memset( &o->meshes[i], 0, sizeof( Mesh ) );
		o->meshCount = first + count;
	}
	if (nthreads < 1) nthreads = 1;
	if (nthreads > count) nthreads = count;
	GeomJob* jobs = (GeomJob*)calloc( nthreads, sizeof( GeomJob ) );
	pthread_t* th = (pthread_t*)calloc( nthreads, sizeof( pthread_t ) );
	for (int t = 0; t < nthreads; t++)
	{
		jobs[t] = (GeomJob){ o, first, count, tris, counts, t, nthreads };
		if (nthreads > 1) pthread_create( &th[t], 0, geom_worker, &jobs[t] ); else geom_worker( &jobs[t] );
	}
	if (nthreads > 1) for (int t = 0; t < nthreads; t++) pthread_join( th[t], 0 );
	free( jobs ); free( th );
}

/* mat4::Inverted, RenderSystem/common_types.h:586-628 (MESA formula) */
void orc_mat4_inverse( const float* c, float* out )
{
	const float inv[16] = {
		c[5] * c[10] * c[15] - c[5] * c[11] * c[14] - c[9] * c[6] * c[15] + c[9] * c[7] * c[14] + c[13] * c[6] * c[11] - c[13] * c[7] * c[10],
		-c[1] * c[10] * c[15] + c[1] * c[11] * c[14] + c[9] * c[2] * c[15] - c[9] * c[3] * c[14] - c[13] * c[2] * c[11] + c[13] * c[3] * c[10],
		c[1] * c[6] * c[15] - c[1] * c[7] * c[14] - c[5] * c[2] * c[15] + c[5] * c[3] * c[14] + c[13] * c[2] * c[7] - c[13] * c[3] * c[6],
		-c[1] * c[6] * c[11] + c[1] * c[7] * c[10] + c[5] * c[2] * c[11] - c[5] * c[3] * c[10] - c[9] * c[2] * c[7] + c[9] * c[3] * c[6],
		-c[4] * c[10] * c[15] + c[4] * c[11] * c[14] + c[8] * c[6] * c[15] - c[8] * c[7] * c[14] - c[12] * c[6] * c[11] + c[12] * c[7] * c[10],
		c[0] * c[10] * c[15] - c[0] * c[11] * c[14] - c[8] * c[2] * c[15] + c[8] * c[3] * c[14] + c[12] * c[2] * c[11] - c[12] * c[3] * c[10],
		-c[0] * c[6] * c[15] + c[0] * c[7] * c[14] + c[4] * c[2] * c[15] - c[4] * c[3] * c[14] - c[12] * c[2] * c[7] + c[12] * c[3] * c[6],
		c[0] * c[6] * c[11] - c[0] * c[7] * c[10] - c[4] * c[2] * c[11] + c[4] * c[3] * c[10] + c[8] * c[2] * c[7] - c[8] * c[3] * c[6],
		c[4] * c[9] * c[15] - c[4] * c[11] * c[13] - c[8] * c[5] * c[15] + c[8] * c[7] * c[13] + c[12] * c[5] * c[11] - c[12] * c[7] * c[9],
		-c[0] * c[9] * c[15] + c[0] * c[11] * c[13] + c[8] * c[1] * c[15] - c[8] * c[3] * c[13] - c[12] * c[1] * c[11] + c[12] * c[3] * c[9],
		c[0] * c[5] * c[15] - c[0] * c[7] * c[13] - c[4] * c[1] * c[15] + c[4] * c[3] * c[13] + c[12] * c[1] * c[7] - c[12] * c[3] * c[5],
		-c[0] * c[5] * c[11] + c[0] * c[7] * c[9] + c[4] * c[1] * c[11] - c[4] * c[3] * c[9] - c[8] * c[1] * c[7] + c[8] * c[3] * c[5],
		-c[4] * c[9] * c[14] + c[4] * c[10] * c[13] + c[8] * c[5] * c[14] - c[8] * c[6] * c[13] - c[12] * c[5] * c[10] + c[12] * c[6] * c[9],
		c[0] * c[9] * c[14] - c[0] * c[10] * c[13] - c[8] * c[1] * c[14] + c[8] * c[2] * c[13] + c[12] * c[1] * c[10] - c[12] * c[2] * c[9],
		-c[0] * c[5] * c[14] + c[0] * c[6] * c[13] + c[4] * c[1] * c[14] - c[4] * c[2] * c[13] - c[12] * c[1] * c[6] + c[12] * c[2] * c[5],
		c[0] * c[5] * c[10] - c[0] * c[6] * c[9] - c[4] * c[1] * c[10] + c[4] * c[2] * c[9] + c[8] * c[1] * c[6] - c[8] * c[2] * c[5] };
	const float det = c[0] * inv[0] + c[1] * inv[4] + c[2] * inv[8] + c[3] * inv[12];
	if (det != 0)
	{
		const float invdet = 1.0f / det;
		for (int i = 0; i < 16; i++) out[i] = inv[i] * invdet;
	}
	else
	{
		for (int i = 0; i < 16; i++) out[i] = (i % 5 == 0) ? 1.0f : 0.0f;
	}
}

/* instance-space ray: mat4::TransformPoint / TransformVector (common_types.h:633-651),
   affine (w == 1); the direction is NOT renormalised so t stays in world units. */
static inline f3 xform_point( const float* c, f3 v ) { return mk3( c[0] * v.x + c[1] * v.y + c[2] * v.z + c[3], c[4] * v.x + c[5] * v.y + c[6] * v.z + c[7], c[8] * v.x + c[9] * v.y + c[10] * v.z + c[11] ); }
static inline f3 xform_vector( const float* c, f3 v ) { return mk3( c[0] * v.x + c[1] * v.y + c[2] * v.z, c[4] * v.x + c[5] * v.y + c[6] * v.z, c[8] * v.x + c[9] * v.y + c[10] * v.z ); }

/* RenderCore::SetInstance, OptixPrime_B/rendercore.cpp:229-243 */
void orc_set_instance( Oracle* o, int instIdx, int meshIdx, const float* m16 )
{
	if (meshIdx == -1) { if (o->instCount > instIdx) o->instCount = instIdx; return; }
	if (instIdx >= o->instCap)
	{
		o->instCap = instIdx + 16;
		o->inst = (Instance*)realloc( o->inst, sizeof( Instance ) * o->instCap );
	}
	if (instIdx >= o->instCount) o->instCount = instIdx + 1;
	o->inst[instIdx].mesh = meshIdx;
	memcpy( o->inst[instIdx].T, m16, 64 );
}

/* RenderCore::UpdateToplevel (rendercore.cpp:250-270) + instance descriptors (:481-505) */
void orc_update_toplevel( Oracle* o )
{
	for (int i = 0; i < o->instCount; i++)
	{
		Instance* in = &o->inst[i];
		orc_mat4_inverse( in->T, in->inv );
		const Mesh* m = &o->meshes[in->mesh];
		in->wmin = s3( FLT_MAX ), in->wmax = s3( -FLT_MAX );
		if (m->triCount == 0) continue;
		for (int k = 0; k < 8; k++)
		{
			const f3 c = mk3( (k & 1) ? m->aabbMax.x : m->aabbMin.x, (k & 2) ? m->aabbMax.y : m->aabbMin.y, (k & 4) ? m->aabbMax.z : m->aabbMin.z );
			const f3 p = xform_point( in->T, c );
			in->wmin = mk3( fminf( in->wmin.x, p.x ), fminf( in->wmin.y, p.y ), fminf( in->wmin.z, p.z ) );
			in->wmax = mk3( fmaxf( in->wmax.x, p.x ), fmaxf( in->wmax.y, p.y ), fmaxf( in->wmax.z, p.z ) );
		}
	}
}

/* ------------------------------------------------------------------------------------- */
/* traversal                                                                               */
/* ------------------------------------------------------------------------------------- */
typedef struct { f3 O, D, invD; float tmin; } TRay;
typedef struct { float t; int tri, inst; float u, v; } THit;

static inline float safe_inv( float d ) { return (d > -1e-30f && d < 1e-30f) ? (d < 0 ? -1e30f : 1e30f) : 1.0f / d; }

/* conservative slab test; culling only, never decides a hit (DESIGN.md "Traversal numerics") */
static inline int box_hit( const TRay* r, f3 bmin, f3 bmax, float tmax, float* tnear )
{
	const float t1x = (bmin.x - r->O.x) * r->invD.x, t2x = (bmax.x - r->O.x) * r->invD.x;
	const float t1y = (bmin.y - r->O.y) * r->invD.y, t2y = (bmax.y - r->O.y) * r->invD.y;
	const float t1z = (bmin.z - r->O.z) * r->invD.z, t2z = (bmax.z - r->O.z) * r->invD.z;
	const float tn = fmaxf( fmaxf( fminf( t1x, t2x ), fminf( t1y, t2y ) ), fminf( t1z, t2z ) );
	const float tf = fminf( fminf( fmaxf( t1x, t2x ), fmaxf( t1y, t2y ) ), fmaxf( t1z, t2z ) );
	*tnear = tn;
	const float tfp = tf * 1.00001f + 1e-30f;
	return tn <= tfp && tfp >= r->tmin && tn <= tmax * 1.00001f + 1e-30f;
}

/* Möller–Trumbore, after RenderCore_Bart/common.h:19-50 with the open interval (tmin, tmax)
   of OptiX Prime's ray format (optix_prime_declarations.h:76) and an exact-zero determinant
   test.  Here u weights vertex1, v weights vertex2 (w = 1-u-v weights vertex0); trace_ray
   converts the final hit to the Prime convention (to_prime_bary). */
static inline int intersect_tri( const TRay* r, const lh2_CoreTri* tri, float* t, float* uo, float* vo )
{
	const f3 v0 = lf3( tri->vertex0 ), v1 = lf3( tri->vertex1 ), v2 = lf3( tri->vertex2 );
	const f3 e1 = sub3( v1, v0 ), e2 = sub3( v2, v0 );
	const f3 h = cross3( r->D, e2 );
	const float a = dot3( e1, h );
	if (a == 0.0f) return 0;
	const float f = 1.0f / a;
	const f3 s = sub3( r->O, v0 );
	const float u = f * dot3( s, h );
	if (u < 0.0f || u > 1.0f) return 0;
	const f3 q = cross3( s, e1 );
	const float v = f * dot3( r->D, q );
	if (v < 0.0f || u + v > 1.0f) return 0;
	*t = f * dot3( e2, q );
	*uo = u, *vo = v;
	return 1;
}

static inline int better( float t, int inst, int tri, const THit* b )
{
	if (t < b->t) return 1;
	if (t > b->t) return 0;
	return inst < b->inst || (inst == b->inst && tri < b->tri);
}

/* returns 1 if (any-hit mode) an occluder was found */
static int traverse_blas( const Mesh* m, const TRay* r, int instIdx, THit* best, int anyHit, uint32_t* nodes, uint32_t* ttests )
{
	if (m->triCount == 0) return 0;
	int stack[256]; float stackT[256]; int sp = 0;
	float tn;
	(*nodes)++;
	if (!box_hit( r, m->pool[0].bmin, m->pool[0].bmax, best->t, &tn )) return 0;
	int cur = 0;
	while (1)
	{
		const BNode* n = &m->pool[cur];
		if (n->count > 0)
		{
			for (int i = n->first; i < n->first + n->count; i++)
			{
				const int ti = m->idx[i];
				float t, u, v;
				(*ttests)++;
				if (intersect_tri( r, &m->tris[ti], &t, &u, &v ) && t > r->tmin)
				{
					if (anyHit) { if (t < best->t) return 1; continue; }
					if (better( t, instIdx, ti, best )) best->t = t, best->tri = ti, best->inst = instIdx, best->u = u, best->v = v;
				}
			}
		}
		else
		{
			const int c0 = n->first, c1 = n->first + 1;
			float tn0, tn1;
			*nodes += 2;
			const int h0 = box_hit( r, m->pool[c0].bmin, m->pool[c0].bmax, best->t, &tn0 );
			const int h1 = box_hit( r, m->pool[c1].bmin, m->pool[c1].bmax, best->t, &tn1 );
			if (h0 && h1)
			{
				if (sp >= 256) abort();
				if (tn1 < tn0) { stack[sp] = c0; stackT[sp++] = tn0; cur = c1; } else { stack[sp] = c1; stackT[sp++] = tn1; cur = c0; }
				continue;
			}
			if (h0) { cur = c0; continue; }
			if (h1) { cur = c1; continue; }
		}
		/* pop, culling entries whose entry distance exceeds the current best */
		int found = 0;
		while (sp)
		{
			--sp;
			if (stackT[sp] <= best->t * 1.00001f + 1e-30f) { cur = stack[sp]; found = 1; break; }
		}
		if (!found) break;
	}
	return 0;
}

/* Hit-record barycentrics in the OptiX Prime convention the Prime_B shading code assumes
   (material_shared.h:77-78,91-92,105-107 interpolate u*v0 + v*v1 + (1-u-v)*v2; SURVEY.md §7
   "Barycentric convention"): u = weight of vertex0, v = weight of vertex1.  Möller–Trumbore gives
   the weights of vertex1 and vertex2, so u' = 1 - (u + v), v' = u. */
static inline void to_prime_bary( THit* h ) { const float w = 1.0f - (h->u + h->v); h->v = h->u; h->u = w; }

static void trace_ray( const Oracle* o, f3 O, f3 D, float tmin, float tmax, int anyHit, THit* best, uint32_t* nodes, uint32_t* ttests, int* occluded )
{
	best->t = tmax, best->tri = -1, best->inst = -1, best->u = best->v = 0;
	*occluded = 0;
	for (int i = 0; i < o->instCount; i++)
	{
		const Instance* in = &o->inst[i];
		TRay wr;
		wr.O = O, wr.D = D, wr.tmin = tmin;
		wr.invD = mk3( safe_inv( D.x ), safe_inv( D.y ), safe_inv( D.z ) );
		float tn;
		if (!box_hit( &wr, in->wmin, in->wmax, best->t, &tn )) continue;
		TRay r;
		r.O = xform_point( in->inv, O );
		r.D = xform_vector( in->inv, D );
		r.tmin = tmin;
		r.invD = mk3( safe_inv( r.D.x ), safe_inv( r.D.y ), safe_inv( r.D.z ) );
		if (traverse_blas( &o->meshes[in->mesh], &r, i, best, anyHit, nodes, ttests )) { *occluded = 1; return; }
	}
	if (best->tri >= 0) to_prime_bary( best );
}

/* ------------------------------------------------------------------------------------- */
/* materials: RenderCore::SetMaterials (rendercore.cpp:353-399)                             */
/* ------------------------------------------------------------------------------------- */
static inline uint32_t TOCHAR( float a ) { return lh2_f2u( a * 255.0f ); }
static inline uint32_t TOUINT4( float a, float b, float c, float d ) { return TOCHAR( a ) + (TOCHAR( b ) << 8) + (TOCHAR( c ) << 16) + (TOCHAR( d ) << 24); }
#define HASSMOOTHNORMALS (1 << 11)
#define HASALPHA (1 << 12)
#define ISDIELECTRIC (1 << 0)
void orc_set_materials( Oracle* o, const lh2_CoreMaterial* mat, int n )
{
	free( o->mats );
	o->mats = (Mat*)calloc( n ? n : 1, sizeof( Mat ) );
	o->matCount = n;
	for (int i = 0; i < n; i++)
	{
		const lh2_CoreMaterial* m = &mat[i];
		Mat* g = &o->mats[i];
		g->diffuse[0] = lh2_f2h( m->color.value.x ), g->diffuse[1] = lh2_f2h( m->color.value.y ), g->diffuse[2] = lh2_f2h( m->color.value.z );
		g->transmittance[0] = lh2_f2h( 1 - m->absorption.value.x );
		g->transmittance[1] = lh2_f2h( 1 - m->absorption.value.y );
		g->transmittance[2] = lh2_f2h( 1 - m->absorption.value.z );
		g->params[0] = TOUINT4( m->metallic.value, m->subsurface.value, m->specular.value, m->roughness.value );
		g->params[1] = TOUINT4( m->specularTint.value, m->anisotropic.value, m->sheen.value, m->sheenTint.value );
		g->params[2] = TOUINT4( m->clearcoat.value, m->clearcoatGloss.value, m->transmission.value, 0 );
		g->params[3] = fbits( m->eta.value );
		/* maps: RenderCore::Map (rendercore.h:79-86) for each textured field (rendercore.cpp:379-384) */
		const struct { int id; lh2_float2 sc, of; int slot; uint32_t flag; } F[6] = {
			{ m->color.textureID, m->color.uvscale, m->color.uvoffset, 0, 1u << 2 },
			{ m->detailColor.textureID, m->detailColor.uvscale, m->detailColor.uvoffset, 1, 1u << 9 },
			{ m->normals.textureID, m->normals.uvscale, m->normals.uvoffset, 2, 1u << 3 },
			{ m->detailNormals.textureID, m->detailNormals.uvscale, m->detailNormals.uvoffset, 3, 1u << 7 },
			{ m->specular.textureID, m->specular.uvscale, m->specular.uvoffset, 4, 1u << 4 },
			{ m->roughness.textureID, m->roughness.uvscale, m->roughness.uvoffset, 5, 1u << 5 } };
		uint32_t tf = 0;
		for (int k = 0; k < 6; k++)
		{
			if (F[k].id == -1) continue;
			if (F[k].id < 0 || F[k].id >= o->texCount) continue;   /* the core rejects this (FatalError) */
			const lh2_CoreTexDesc* t = &o->tex[F[k].id];
			uint32_t* r = g->maps[F[k].slot];
			r[0] = (t->width & 0xffffu) | ((t->height & 0xffffu) << 16);
			r[1] = (uint32_t)lh2_f2h( F[k].sc.x ) | ((uint32_t)lh2_f2h( F[k].sc.y ) << 16);
			r[2] = (uint32_t)lh2_f2h( F[k].of.x ) | ((uint32_t)lh2_f2h( F[k].of.y ) << 16);
			r[3] = t->firstPixel;
			tf |= F[k].flag;
		}
		/* DIFFUSEMAPISHDR (bit 1) is never read while shading; the reference's test at
		   rendercore.cpp:386 indexes texDescs[-1] for untextured materials */
		if (m->color.textureID >= 0 && m->color.textureID < o->texCount && (o->tex[m->color.textureID].flags & 8)) tf |= 1u << 1;
		g->flags = (m->eta.value < 1 ? ISDIELECTRIC : 0) + ((m->flags & 1) ? HASSMOOTHNORMALS : 0) + ((m->flags & 2) ? HASALPHA : 0) + tf;
	}
}

/* RenderCore::SetTextures + SyncStorageType (rendercore.cpp:276-336): per storage type, one
   continuous texel array in descriptor order (at least 16 texels); ARGB128 texels are not read
   by this core's shading and are not kept */
void orc_set_textures( Oracle* o, const lh2_CoreTexDesc* t, int n )
{
	free( o->tex ); free( o->argb32 ); free( o->nrm32 );
	o->tex = (lh2_CoreTexDesc*)calloc( n > 0 ? n : 1, sizeof( lh2_CoreTexDesc ) );
	if (n > 0) memcpy( o->tex, t, sizeof( lh2_CoreTexDesc ) * n );
	o->texCount = n > 0 ? n : 0;
	for (int storage = 0; storage < 3; storage += 2)
	{
		uint32_t total = 0, at = 0;
		for (int i = 0; i < o->texCount; i++) if (o->tex[i].storage == storage) total += o->tex[i].pixelCount;
		const uint32_t cnt = total < 16 ? 16 : total;
		uint32_t* buf = (uint32_t*)calloc( cnt, 4 );
		for (int i = 0; i < o->texCount; i++) if (o->tex[i].storage == storage)
		{
			memcpy( buf + at, o->tex[i].idata, (size_t)o->tex[i].pixelCount * 4 );
			o->tex[i].firstPixel = at, at += o->tex[i].pixelCount;
		}
		if (storage == 0) o->argb32 = buf, o->argb32Count = cnt; else o->nrm32 = buf, o->nrm32Count = cnt;
	}
	for (int i = 0; i < o->texCount; i++) if (o->tex[i].storage == 1)
	{
		uint32_t at = 0;
		for (int j = 0; j < i; j++) if (o->tex[j].storage == 1) at += o->tex[j].pixelCount;
		o->tex[i].firstPixel = at;
	}
}

void orc_set_lights( Oracle* o, const lh2_CoreLightTri* a, int na, const lh2_CorePointLight* p, int np,
	const lh2_CoreSpotLight* s, int ns, const lh2_CoreDirectionalLight* d, int nd )
{
	free( o->area ); free( o->point ); free( o->spot ); free( o->dirl );
	o->area = (lh2_CoreLightTri*)malloc( sizeof( *a ) * (na ? na : 1) ); memcpy( o->area, a, sizeof( *a ) * na ); o->nArea = na;
	o->point = (lh2_CorePointLight*)malloc( sizeof( *p ) * (np ? np : 1) ); memcpy( o->point, p, sizeof( *p ) * np ); o->nPoint = np;
	o->spot = (lh2_CoreSpotLight*)malloc( sizeof( *s ) * (ns ? ns : 1) ); memcpy( o->spot, s, sizeof( *s ) * ns ); o->nSpot = ns;
	o->dirl = (lh2_CoreDirectionalLight*)malloc( sizeof( *d ) * (nd ? nd : 1) ); memcpy( o->dirl, d, sizeof( *d ) * nd ); o->nDir = nd;
}

void orc_set_sky( Oracle* o, const float* rgb, int w, int h )
{
	free( o->sky );
	o->sky = (float*)malloc( sizeof( float ) * 3 * ((w * h) > 0 ? w * h : 1) );
	memcpy( o->sky, rgb, sizeof( float ) * 3 * w * h );
	o->skyW = w, o->skyH = h;
}

void orc_setting( Oracle* o, const char* name, float value ) /* rendercore.cpp:439-457 */
{
	if (!strcmp( name, "epsilon" )) o->geometryEpsilon = value;
	else if (!strcmp( name, "clampValue" )) o->clampValue = value;
	else if (!strcmp( name, "maxPathLength" )) orc_set_max_path_length( o, (int)value );
	else if (!strcmp( name, "primeRef" )) o->primeRef = value != 0;
}

void orc_set_target( Oracle* o, int w, int h, int spp ) /* rendercore.cpp:149-209 */
{
	o->w = w, o->h = h, o->spp = spp;
	free( o->acc );
	o->acc = (float*)calloc( (size_t)w * h * 4, sizeof( float ) );
	o->samplesTaken = 0;
}

void orc_set_probe( Oracle* o, int x, int y ) { o->probeX = x, o->probeY = y; }
/* diagnostics: log the path vertices and shadow rays of pixel px (-1: none) of the next renders */
void orc_debug_pixel( Oracle* o, int px, int cap )
{
	free( o->debugLog );
	o->debugPixel = px, o->debugCount = 0, o->debugCap = px >= 0 ? cap : 0;
	o->debugLog = px >= 0 ? (float*)calloc( (size_t)cap * 16, sizeof( float ) ) : 0;
}
int orc_debug_log( const Oracle* o, float* out, int cap )
{
	int n = o->debugCount < o->debugCap ? o->debugCount : o->debugCap;
	if (n > cap) n = cap;
	if (n > 0) memcpy( out, o->debugLog, (size_t)n * 16 * sizeof( float ) );
	return n;
}

/* ------------------------------------------------------------------------------------- */
/* tools: tools_shared.h                                                                   */
/* ------------------------------------------------------------------------------------- */
static inline uint32_t PackNormal( f3 N ) /* tools_shared.h:101-112 */
{
	const float f = 65535.0f / fmaxf( sqrtf( 8.0f * N.z + 8.0f ), 0.0001f );
	return lh2_f2u( N.x * f + 32767.0f ) + (lh2_f2u( N.y * f + 32767.0f ) << 16);
}
static inline f3 UnpackNormal( uint32_t p ) /* tools_shared.h:113-120 */
{
	float nx = (float)(p & 65535) * (2.0f / 65535.0f), ny = (float)(p >> 16) * (2.0f / 65535.0f), nz = 0, nw = 0;
	nx = nx + -1.0f, ny = ny + -1.0f, nz = nz + 1.0f, nw = nw + -1.0f;
	float l = nx * -nx + ny * -ny + nz * -nw;
	nz = l, l = sqrtf( l ), nx *= l, ny *= l;
	return mk3( nx * 2.0f + 0.0f, ny * 2.0f + 0.0f, nz * 2.0f + -1.0f );
}
static inline f3 SampleSkydome( const Oracle* o, f3 D ) /* tools_shared.h:185-192 */
{
	const uint32_t u = lh2_f2u( (float)o->skyW * 0.5f * (1.0f + lh2_atan2f( D.x, -D.z ) * INVPI) );
	const uint32_t v = lh2_f2u( (float)o->skyH * lh2_acosf( D.y ) * INVPI );
	const uint32_t idx = u + v * (uint32_t)o->skyW;
	if (idx < (uint32_t)(o->skyW * o->skyH)) return mk3( o->sky[idx * 3], o->sky[idx * 3 + 1], o->sky[idx * 3 + 2] );
	return s3( 0 );
}
static inline float SurvivalProbability( f3 a ) { return fminf( 1.0f, fmaxf( fmaxf( a.x, a.y ), a.z ) ); }
static inline f3 SafeOrigin( f3 O, f3 R, f3 N, float eps ) /* tools_shared.h:279-292 */
{
	const float parallel = 1 - fabsf( dot3( N, R ) );
	const float v = parallel * parallel;
	const float side = 1.0f;
	return add3( add3( O, muls( muls( R, eps ), 1 - v ) ), muls( muls( muls( N, side ), eps ), v ) );
}
static inline f3 ConsistentNormal( f3 D, f3 iN, float alpha ) /* tools_shared.h:296-310 */
{
	const float t = PI - 2 * alpha, q = (t * t) / (PI * (PI + (2 * PI - 4) * alpha));
	const float b = dot3( D, iN ), g = 1 + q * (b - 1), rho = sqrtf( q * (1 + g) / (1 + b) );
	const f3 Rc = sub3( muls( iN, g + rho * b ), smul( rho, D ) );
	return normalize3( add3( D, Rc ) );
}
static inline f3 World2Tangent( f3 V, f3 N, f3 T, f3 B ) { return mk3( dot3( V, T ), dot3( V, B ), dot3( V, N ) ); }
static inline f3 Tangent2World( f3 V, f3 N, f3 T, f3 B ) { return add3( add3( smul( V.x, T ), smul( V.y, B ) ), smul( V.z, N ) ); }
static inline f3 DiffuseReflectionCosWeighted( float r0, float r1 ) /* tools_shared.h:250-256 */
{
	const float term1 = TWOPI * r0, term2 = sqrtf( 1 - r1 );
	float s, c;
	lh2_sincosf( term1, &s, &c );
	return mk3( c * term2, s * term2, sqrtf( r1 ) );
}

/* ------------------------------------------------------------------------------------- */
/* shading data: material_shared.h:19-178 (OPTIXPRIMEBUILD, CONSISTENTNORMALS, no textures)*/
/* ------------------------------------------------------------------------------------- */
typedef struct
{
	f3 color; int flags;
	f3 transmittance; int matID;
	f4 tint;
	uint32_t params[4];
} ShadingData;
#define CHAR2FLT(a,s) (((float)(((a)>>s)&255))*(1.0f/255.0f))
#define METALLIC CHAR2FLT( sd->params[0], 0 )
#define SUBSURFACE CHAR2FLT( sd->params[0], 8 )
#define SPECULAR CHAR2FLT( sd->params[0], 16 )
#define ROUGHNESS (fmaxf( 0.001f, CHAR2FLT( sd->params[0], 24 ) ))
#define SPECTINT CHAR2FLT( sd->params[1], 0 )
#define ANISOTROPIC CHAR2FLT( sd->params[1], 8 )
#define SHEEN CHAR2FLT( sd->params[1], 16 )
#define SHEENTINT CHAR2FLT( sd->params[1], 24 )
#define CLEARCOAT CHAR2FLT( sd->params[2], 0 )
#define CLEARCOATGLOSS CHAR2FLT( sd->params[2], 8 )
#define TRANSMISSION CHAR2FLT( sd->params[2], 16 )
#define TINT f4xyz( sd->tint )
#define LUMINANCE sd->tint.w
#define ETA bitsf( sd->params[3] )

static inline f3 linear_rgb_to_ciexyz( f3 rgb )
{
	return mk3( fmaxf( 0.0f, 0.412453f * rgb.x + 0.357580f * rgb.y + 0.180423f * rgb.z ),
		fmaxf( 0.0f, 0.212671f * rgb.x + 0.715160f * rgb.y + 0.072169f * rgb.z ),
		fmaxf( 0.0f, 0.019334f * rgb.x + 0.119193f * rgb.y + 0.950227f * rgb.z ) );
}
static inline f3 ciexyz_to_linear_rgb( f3 xyz )
{
	return mk3( fmaxf( 0.0f, 3.240479f * xyz.x - 1.537150f * xyz.y - 0.498535f * xyz.z ),
		fmaxf( 0.0f, -0.969256f * xyz.x + 1.875992f * xyz.y + 0.041556f * xyz.z ),
		fmaxf( 0.0f, 0.055648f * xyz.x - 0.204043f * xyz.y + 1.057311f * xyz.z ) );
}

/* texel fetch: sampling_shared.h:35-86 with BILINEAR (core_settings.h:31), MIPLEVELCOUNT 5
   (common_settings.h:49).  The reference leaves three cases undefined; here (and in the core):
   float->int conversions saturate (lh2_f2i), a MIP level narrower than one texel counts as one
   texel (the reference takes % 0 there), and texel indices are clamped to the array. */
#define MIPLEVELCOUNT 5
static inline f4 texel_u8( uint32_t v )   /* __uchar4_to_float4: x = lowest byte */
{
	const float r = 1.0f / 256.0f;
	f4 t;
	t.x = (float)(v & 255u) * r, t.y = (float)((v >> 8) & 255u) * r, t.z = (float)((v >> 16) & 255u) * r, t.w = (float)(v >> 24) * r;
	return t;
}
static f4 FetchTexel( const uint32_t* tex, uint32_t count, f2 tc, int o, int w, int h )
{
	if (w < 1) w = 1;
	if (h < 1) h = 1;
	const float tcx = (fmaxf( tc.x + 1000, 0.0f ) * (float)w) - 0.5f;
	const float tcy = (fmaxf( tc.y + 1000, 0.0f ) * (float)h) - 0.5f;
	const int iu = lh2_f2i( tcx ) % w, iv = lh2_f2i( tcy ) % h;
	const float fu = tcx - floorf( tcx ), fv = tcy - floorf( tcy );
	const float w0 = (1 - fu) * (1 - fv), w1 = fu * (1 - fv), w2 = (1 - fu) * fv, w3 = 1 - (w0 + w1 + w2);
	const uint32_t iu1 = (uint32_t)((iu + 1) % w), iv1 = (uint32_t)((iv + 1) % h);
	uint32_t a[4] = { (uint32_t)o + (uint32_t)iu + (uint32_t)iv * (uint32_t)w, (uint32_t)o + iu1 + (uint32_t)iv * (uint32_t)w,
		(uint32_t)o + (uint32_t)iu + iv1 * (uint32_t)w, (uint32_t)o + iu1 + iv1 * (uint32_t)w };
	f4 p[4];
	for (int k = 0; k < 4; k++) p[k] = texel_u8( tex[a[k] < count ? a[k] : count - 1] );
	f4 r;
	r.x = p[0].x * w0 + p[1].x * w1 + p[2].x * w2 + p[3].x * w3;
	r.y = p[0].y * w0 + p[1].y * w1 + p[2].y * w2 + p[3].y * w3;
	r.z = p[0].z * w0 + p[1].z * w1 + p[2].z * w2 + p[3].z * w3;
	r.w = p[0].w * w0 + p[1].w * w1 + p[2].w * w2 + p[3].w * w3;
	return r;
}
static f4 FetchTexelTrilinear( const uint32_t* tex, uint32_t count, float lambda, f2 tc, int offset, int width, int height )
{
	int level0 = lh2_f2i( lambda );
	if (level0 > MIPLEVELCOUNT - 1) level0 = MIPLEVELCOUNT - 1;
	const int level1 = level0 + 1 > MIPLEVELCOUNT - 1 ? MIPLEVELCOUNT - 1 : level0 + 1;
	const float f = lambda - floorf( lambda );
	int o0 = offset, w0 = width, h0 = height;
	for (int i = 0; i < level0; i++) o0 += w0 * h0, w0 >>= 1, h0 >>= 1;
	int o1 = offset, w1 = width, h1 = height;
	for (int i = 0; i < level1; i++) o1 += w1 * h1, w1 >>= 1, h1 >>= 1;
	const f4 p0 = FetchTexel( tex, count, tc, o0, w0, h0 ), p1 = FetchTexel( tex, count, tc, o1, w1, h1 );
	f4 r;
	r.x = (1 - f) * p0.x + f * p1.x, r.y = (1 - f) * p0.y + f * p1.y, r.z = (1 - f) * p0.z + f * p1.z, r.w = (1 - f) * p0.w + f * p1.w;
	return r;
}
/* uvscale * (uvoffs + (tu, tv)) with the halves of a map record */
static inline f2 MapCoord( const uint32_t* m, float tu, float tv )
{
	f2 c;
	c.x = lh2_h2f( (uint16_t)(m[1] & 0xffff) ) * (lh2_h2f( (uint16_t)(m[2] & 0xffff) ) + tu);
	c.y = lh2_h2f( (uint16_t)(m[1] >> 16) ) * (lh2_h2f( (uint16_t)(m[2] >> 16) ) + tv);
	return c;
}
static inline f4 MapFetch( const uint32_t* tex, uint32_t count, const uint32_t* m, float tu, float tv )
{
	return FetchTexel( tex, count, MapCoord( m, tu, tv ), (int)m[3], (int)(m[0] & 0xffff), (int)(m[0] >> 16) );
}
int orc_fetch_texel( const Oracle* o, int storage, float u, float v, int offset, int w, int h, float lambda, int trilinear, float* out4 )
{
	const uint32_t* tex = storage == 2 ? o->nrm32 : o->argb32;
	const uint32_t cnt = storage == 2 ? o->nrm32Count : o->argb32Count;
	if (!tex) return -1;
	f2 tc; tc.x = u, tc.y = v;
	const f4 r = trilinear ? FetchTexelTrilinear( tex, cnt, lambda, tc, offset, w, h ) : FetchTexel( tex, cnt, tc, offset, w, h );
	out4[0] = r.x, out4[1] = r.y, out4[2] = r.z, out4[3] = r.w;
	return 0;
}

static void GetShadingData( const Oracle* o, f3 D, float u, float v, float coneWidth, const lh2_CoreTri* tri, int instIdx,
	ShadingData* sd, f3* N, f3* iN, f3* fN, f3* T )
{
	const Mat* mat = &o->mats[tri->material];
	sd->color = mk3( lh2_h2f( mat->diffuse[0] ), lh2_h2f( mat->diffuse[1] ), lh2_h2f( mat->diffuse[2] ) );
	sd->flags = 0;
	sd->transmittance = mk3( lh2_h2f( mat->transmittance[0] ), lh2_h2f( mat->transmittance[1] ), lh2_h2f( mat->transmittance[2] ) );
	sd->matID = 0;
	memcpy( sd->params, mat->params, 16 );
	const f3 tint_xyz = linear_rgb_to_ciexyz( sd->color );
	const f3 tnt = tint_xyz.y > 0 ? ciexyz_to_linear_rgb( muls( tint_xyz, 1.0f / tint_xyz.y ) ) : s3( 1 );
	sd->tint.x = tnt.x, sd->tint.y = tnt.y, sd->tint.z = tnt.z, sd->tint.w = tint_xyz.y;
	const uint32_t flags = mat->flags;
	*N = *iN = *fN = mk3( tri->Nx, tri->Ny, tri->Nz );
	*T = lf3( tri->T );
	const float w = 1 - (u + v);
	if (flags & HASSMOOTHNORMALS)
		*iN = normalize3( add3( add3( smul( u, lf3( tri->vN0 ) ), smul( v, lf3( tri->vN1 ) ) ), smul( w, lf3( tri->vN2 ) ) ) );
	const float* inv = o->inst[instIdx].inv;
	const f3 A = mk3( inv[0], inv[1], inv[2] ), B = mk3( inv[4], inv[5], inv[6] ), C = mk3( inv[8], inv[9], inv[10] );
	const f3 n0 = *N, i0 = *iN;
	*N = add3( add3( smul( n0.x, A ), smul( n0.y, B ) ), smul( n0.z, C ) );
	*iN = add3( add3( smul( i0.x, A ), smul( i0.y, B ) ), smul( i0.z, C ) );
	const int backSide = dot3( D, *N ) > 0;
	const float alpha = u * tri->alpha.x + v * tri->alpha.y + w * tri->alpha.z;
	*iN = smul( backSide ? -1.0f : 1.0f, ConsistentNormal( muls( D, -1.0f ), backSide ? muls( *iN, -1.0f ) : *iN, alpha ) );
	*fN = *iN;
	/* texturing: material_shared.h:99-171 (OPTIXPRIMEBUILD barycentrics) */
	if (!(flags & ((1u << 2) | (1u << 9) | (1u << 4) | (1u << 3) | (1u << 7) | (1u << 5)))) return;
	const float tu = u * tri->u0 + v * tri->u1 + w * tri->u2;
	const float tv = u * tri->v0 + v * tri->v1 + w * tri->v2;
	if (flags & (1u << 2))   /* HASDIFFUSEMAP */
	{
		const float lambda = tri->LOD + lh2_log2f( coneWidth * (1.0f / fabsf( dot3( D, *N ) )) );   /* eq. 26 */
		const uint32_t* m = mat->maps[0];
		const f4 texel = FetchTexelTrilinear( o->argb32, o->argb32Count, lambda, MapCoord( m, tu, tv ), (int)m[3], (int)(m[0] & 0xffff), (int)(m[0] >> 16) );
		if ((flags & HASALPHA) && texel.w < 0.5f)
		{
			sd->flags |= 1;
			return;
		}
		sd->color = mul3( sd->color, mk3( texel.x, texel.y, texel.z ) );
		if (flags & (1u << 9))   /* HAS2NDDIFFUSEMAP */
		{
			const f4 t1 = MapFetch( o->argb32, o->argb32Count, mat->maps[1], tu, tv );
			sd->color = add3( sd->color, sub3( mk3( t1.x, t1.y, t1.z ), s3( 0.5f ) ) );
		}
	}
	if (flags & (1u << 3))   /* HASNORMALMAP */
	{
		const f3 Bt = lf3( tri->B );
		/* part3 = baseData.z = transmittance_g | transmittance_b << 16 (CUDAMaterial layout) */
		const uint32_t part3 = (uint32_t)mat->transmittance[1] | ((uint32_t)mat->transmittance[2] << 16);
		const float b0 = (float)((part3 >> 8) & 255) - 128.0f;
		const float n0scale = copysignf( -0.0001f + 0.0001f * lh2_expf( 0.1f * fabsf( b0 ) ), b0 );
		const f4 t0 = MapFetch( o->nrm32, o->nrm32Count, mat->maps[2], tu, tv );
		f3 sN = mk3( (t0.x - 0.5f) * 2.0f, (t0.y - 0.5f) * 2.0f, (t0.z - 0.5f) * 2.0f );
		sN.x *= n0scale, sN.y *= n0scale;
		if (flags & (1u << 7))   /* HAS2NDNORMALMAP */
		{
			const float b1 = (float)((part3 >> 16) & 255) - 128.0f;
			const float n1scale = copysignf( -0.0001f + 0.0001f * lh2_expf( 0.1f * b1 ), b1 );
			const f4 t1 = MapFetch( o->nrm32, o->nrm32Count, mat->maps[3], tu, tv );
			f3 l1 = mk3( (t1.x - 0.5f) * 2.0f, (t1.y - 0.5f) * 2.0f, (t1.z - 0.5f) * 2.0f );
			l1.x *= n1scale, l1.y *= n1scale;
			sN = add3( sN, l1 );
		}
		sN = normalize3( sN );
		*fN = normalize3( add3( add3( smul( sN.x, *T ), smul( sN.y, Bt ) ), smul( sN.z, *iN ) ) );
	}
	if (flags & (1u << 5))   /* HASROUGHNESSMAP */
	{
		const f4 t = MapFetch( o->argb32, o->argb32Count, mat->maps[5], tu, tv );
		sd->params[0] = (sd->params[0] & 0xffffff) + (lh2_f2u( t.x * 255.0f ) << 24);
	}
}

/* ------------------------------------------------------------------------------------- */
/* lights: lights_shared.h:36-261                                                          */
/* ------------------------------------------------------------------------------------- */
static inline float PotentialAreaLightContribution( const Oracle* o, int idx, f3 O, f3 N, f3 I, f3 bary )
{
	const lh2_CoreLightTri* l = &o->area[idx];
	f3 L = I;
	if (bary.x >= 0)
	{
		const f3 V0 = lf3( l->vertex0 ), V1 = lf3( l->vertex1 ), V2 = lf3( l->vertex2 );
		L = add3( add3( smul( bary.x, V0 ), smul( bary.y, V1 ) ), smul( bary.z, V2 ) );
	}
	L = sub3( L, O );
	const float att = 1.0f / dot3( L, L );
	L = normalize3( L );
	const float LNdotL = fmaxf( 0.0f, -dot3( lf3( l->N ), L ) );
	const float NdotL = fmaxf( 0.0f, dot3( N, L ) );
	return l->energy * LNdotL * NdotL * att;
}
static inline float PotentialPointLightContribution( const Oracle* o, int idx, f3 I, f3 N )
{
	const lh2_CorePointLight* l = &o->point[idx];
	const f3 L = sub3( lf3( l->position ), I );
	const float NdotL = fmaxf( 0.0f, dot3( N, L ) );
	const float att = 1.0f / dot3( L, L );
	return l->energy * NdotL * att;
}
static inline float PotentialSpotLightContribution( const Oracle* o, int idx, f3 I, f3 N )
{
	const lh2_CoreSpotLight* l = &o->spot[idx];
	f3 L = sub3( lf3( l->position ), I );
	const float att = 1.0f / dot3( L, L );
	L = normalize3( L );
	const float d = (fmaxf( 0.0f, -dot3( L, lf3( l->direction ) ) ) - l->cosOuter) / (l->cosInner - l->cosOuter);
	const float NdotL = fmaxf( 0.0f, dot3( N, L ) );
	const float LNdotL = fmaxf( 0.0f, fminf( 1.0f, d ) );
	return (l->radiance.x + l->radiance.y + l->radiance.z) * LNdotL * NdotL * att;
}
static inline float PotentialDirectionalLightContribution( const Oracle* o, int idx, f3 I, f3 N )
{
	const lh2_CoreDirectionalLight* l = &o->dirl[idx];
	(void)I;
	const float LNdotL = fmaxf( 0.0f, -(l->direction.x * N.x + l->direction.y * N.y + l->direction.z * N.z) );
	return l->energy * LNdotL;
}
static inline float CalculateLightPDF( f3 D, float t, float lightArea, f3 lightNormal )
{
	return (t * t) / (-dot3( D, lightNormal ) * lightArea);
}
/* potential of light i (area, point, spot, dir order) from position I with normal N */
static inline float potential_i( const Oracle* o, int i, f3 I, f3 N, f3 bary, f3 areaI )
{
	if (i < o->nArea) return PotentialAreaLightContribution( o, i, I, N, areaI, bary );
	i -= o->nArea;
	if (i < o->nPoint) return PotentialPointLightContribution( o, i, I, N );
	i -= o->nPoint;
	if (i < o->nSpot) return PotentialSpotLightContribution( o, i, I, N );
	i -= o->nSpot;
	return PotentialDirectionalLightContribution( o, i, I, N );
}
static float LightPickProb( const Oracle* o, int idx, f3 O, f3 N, f3 I ) /* lights_shared.h:123-138 */
{
	const int nl = o->nArea + o->nPoint + o->nSpot + o->nDir;
	float sum = 0, pidx = 0;
	for (int i = 0; i < nl; i++)
	{
		/* area lights: PotentialAreaLightContribution(i, O, N, I, (-1,-1,-1)); others (i, O, N) */
		const float c = potential_i( o, i, O, N, s3( -1 ), I );
		if (i == idx) pidx = c;
		sum += c;
	}
	if (sum <= 0) return 0;
	if (idx < 0 || idx >= o->nArea) return 0; /* Q3 */
	return pidx / sum;
}
static f3 RandomBarycentrics( float r0 ) /* lights_shared.h:145-164 */
{
	const uint32_t uf = lh2_f2u( r0 * 4294967296.0f );
	f2 A = { 1, 0 }, B = { 0, 1 }, C = { 0, 0 };
	for (int i = 0; i < 16; ++i)
	{
		const int d = (uf >> (2 * (15 - i))) & 0x3;
		f2 An, Bn, Cn;
		switch (d)
		{
		case 0: An.x = (B.x + C.x) * 0.5f, An.y = (B.y + C.y) * 0.5f; Bn.x = (A.x + C.x) * 0.5f, Bn.y = (A.y + C.y) * 0.5f; Cn.x = (A.x + B.x) * 0.5f, Cn.y = (A.y + B.y) * 0.5f; break;
		case 1: An = A; Bn.x = (A.x + B.x) * 0.5f, Bn.y = (A.y + B.y) * 0.5f; Cn.x = (A.x + C.x) * 0.5f, Cn.y = (A.y + C.y) * 0.5f; break;
		case 2: An.x = (B.x + A.x) * 0.5f, An.y = (B.y + A.y) * 0.5f; Bn = B; Cn.x = (B.x + C.x) * 0.5f, Cn.y = (B.y + C.y) * 0.5f; break;
		default: An.x = (C.x + A.x) * 0.5f, An.y = (C.y + A.y) * 0.5f; Bn.x = (C.x + B.x) * 0.5f, Bn.y = (C.y + B.y) * 0.5f; Cn = C; break;
		}
		A = An, B = Bn, C = Cn;
	}
	const float rx = (A.x + B.x + C.x) * 0.3333333f, ry = (A.y + B.y + C.y) * 0.3333333f;
	return mk3( rx, ry, 1 - rx - ry );
}
static f3 RandomPointOnLight( const Oracle* o, float r0, float r1, f3 I, f3 N, float* pickProb, float* lightPdf, f3* lightColor )
{
	const int nl = o->nArea + o->nPoint + o->nSpot + o->nDir;
	const float lightCount = (float)nl;
	const f3 bary = RandomBarycentrics( r0 );
	float sum = 0, total = 0;
	int lightIdx = 0;
	for (int i = 0; i < nl; i++) sum += potential_i( o, i, I, N, bary, s3( 0 ) );
	if (sum <= 0) { *lightPdf = 0; return s3( 1 ); }
	r1 *= sum;
	for (int i = 0; i < nl; i++)
	{
		total += potential_i( o, i, I, N, bary, s3( 0 ) );
		if (total >= r1) { lightIdx = i; break; }
	}
	*pickProb = potential_i( o, lightIdx, I, N, bary, s3( 0 ) ) / sum;
	{ const int hi = (int)lightCount - 1; lightIdx = lightIdx < 0 ? 0 : lightIdx > hi ? hi : lightIdx; }
	if (lightIdx < o->nArea)
	{
		const lh2_CoreLightTri* l = &o->area[lightIdx];
		*lightColor = lf3( l->radiance );
		const f3 P = add3( add3( smul( bary.x, lf3( l->vertex0 ) ), smul( bary.y, lf3( l->vertex1 ) ) ), smul( bary.z, lf3( l->vertex2 ) ) );
		f3 L = sub3( I, P );
		const float sqDist = dot3( L, L );
		L = normalize3( L );
		const float LNdotL = L.x * l->N.x + L.y * l->N.y + L.z * l->N.z;
		const float reciSolidAngle = sqDist / (l->area * LNdotL);
		*lightPdf = (LNdotL > 0 && dot3( L, N ) < 0) ? reciSolidAngle : 0;
		return P;
	}
	else if (lightIdx < o->nArea + o->nPoint)
	{
		const lh2_CorePointLight* l = &o->point[lightIdx - o->nArea];
		const f3 pos = lf3( l->position );
		*lightColor = lf3( l->radiance ); /* Q2 */
		const f3 L = sub3( I, pos );
		const float sqDist = dot3( L, L );
		*lightPdf = dot3( L, N ) < 0 ? sqDist : 0;
		return pos;
	}
	else if (lightIdx < o->nArea + o->nPoint + o->nSpot)
	{
		const lh2_CoreSpotLight* l = &o->spot[lightIdx - (o->nArea + o->nPoint)];
		const f3 pos = lf3( l->position );
		f3 L = sub3( I, pos );
		const float sqDist = dot3( L, L );
		L = normalize3( L );
		const float d = (fmaxf( 0.0f, L.x * l->direction.x + L.y * l->direction.y + L.z * l->direction.z ) - l->cosOuter) / (l->cosInner - l->cosOuter);
		const float LNdotL = fminf( 1.0f, d );
		*lightPdf = (LNdotL > 0 && dot3( L, N ) < 0) ? (sqDist / LNdotL) : 0;
		*lightColor = lf3( l->radiance );
		return pos;
	}
	else
	{
		const lh2_CoreDirectionalLight* l = &o->dirl[lightIdx - (o->nArea + o->nPoint + o->nSpot)];
		const f3 L = lf3( l->direction );
		*lightColor = lf3( l->radiance );
		const float NdotL = dot3( L, N );
		*lightPdf = NdotL < 0 ? 1 : 0;
		return sub3( I, smul( 1000.0f, L ) );
	}
}

/* unit-level light entry points (the light KATs, tests/test_oracle_kats.py): the functions above, on the lights set by
   orc_set_lights.  Vectors are float[3]. */
float orc_light_potential( const Oracle* o, int i, const float* I, const float* N, const float* bary, const float* areaI )
{
	return potential_i( o, i, mk3( I[0], I[1], I[2] ), mk3( N[0], N[1], N[2] ), mk3( bary[0], bary[1], bary[2] ), mk3( areaI[0], areaI[1], areaI[2] ) );
}
float orc_light_pick_prob( const Oracle* o, int idx, const float* O, const float* N, const float* I )
{
	return LightPickProb( o, idx, mk3( O[0], O[1], O[2] ), mk3( N[0], N[1], N[2] ), mk3( I[0], I[1], I[2] ) );
}
void orc_random_barycentrics( float r0, float* out3 )
{
	const f3 b = RandomBarycentrics( r0 );
	out3[0] = b.x, out3[1] = b.y, out3[2] = b.z;
}
/* out8: the point on the light (x, y, z), pickProb, lightPdf, lightColor (r, g, b); pickProb and lightColor are 0 when
   no light has potential (lightPdf 0: the shade code queues no shadow ray) */
void orc_random_point_on_light( const Oracle* o, float r0, float r1, const float* I, const float* N, float* out8 )
{
	float pickProb = 0, lightPdf = 0;
	f3 color = s3( 0 );
	const f3 P = RandomPointOnLight( o, r0, r1, mk3( I[0], I[1], I[2] ), mk3( N[0], N[1], N[2] ), &pickProb, &lightPdf, &color );
	out8[0] = P.x, out8[1] = P.y, out8[2] = P.z, out8[3] = pickProb, out8[4] = lightPdf, out8[5] = color.x, out8[6] = color.y, out8[7] = color.z;
}

/* ------------------------------------------------------------------------------------- */
/* Disney BSDF: sharedBSDFs/disney.h:33-333, ggxmdf.h:23-243                               */
/* ------------------------------------------------------------------------------------- */
static inline float schlick_fresnel( float u ) { const float m = saturatef_( 1.0f - u ), m2 = sqrf( m ), m4 = sqrf( m2 ); return m4 * m; }
static inline f3 mix_spectra( f3 a, f3 b, float t ) { return add3( smul( 1.0f - t, a ), smul( t, b ) ); }
static inline f3 mix_one_with_spectra( f3 b, float t ) { return sadd( 1.0f - t, smul( t, b ) ); }
static inline f3 mix_spectra_with_one( f3 a, float t ) { return adds( smul( 1.0f - t, a ), t ); }
static inline void microfacet_alpha_from_roughness( float roughness, float anisotropy, float* ax, float* ay )
{
	const float square_roughness = roughness * roughness;
	const float aspect = sqrtf( 1.0f + anisotropy * (anisotropy < 0 ? 0.9f : -0.9f) );
	*ax = fmaxf( 0.001f, square_roughness / aspect );
	*ay = fmaxf( 0.001f, square_roughness * aspect );
}
static inline float clearcoat_roughness( const ShadingData* sd ) { return mixf( 0.1f, 0.001f, CLEARCOATGLOSS ); }
static inline f3 DisneySpecularFresnel( const ShadingData* sd, f3 o, f3 h )
{
	f3 value = mix_one_with_spectra( TINT, SPECTINT );
	value = muls( value, SPECULAR * 0.08f );
	value = mix_spectra( value, sd->color, METALLIC );
	const float cos_oh = fabsf( dot3( o, h ) );
	return mix_spectra_with_one( value, schlick_fresnel( cos_oh ) );
}
static inline f3 DisneyClearcoatFresnel( const ShadingData* sd, f3 o, f3 h )
{
	const float cos_oh = fabsf( dot3( o, h ) );
	return s3( mixf( 0.04f, 1.0f, schlick_fresnel( cos_oh ) ) * 0.25f * CLEARCOAT );
}
static inline int force_above_surface( f3* direction, f3 normal )
{
	const float Eps = 1.0e-4f;
	const float cos_theta = dot3( *direction, normal );
	const float correction = Eps - cos_theta;
	if (correction <= 0) return 0;
	*direction = normalize3( add3( *direction, smul( correction, normal ) ) );
	return 1;
}
static inline float Fr_L( float VDotN, float eio )
{
	if (VDotN < 0.0f) eio = 1.0f / eio, VDotN = fabsf( VDotN );
	const float SinThetaT2 = sqrf( eio ) * (1.0f - VDotN * VDotN);
	if (SinThetaT2 > 1.0f) return 1.0f;
	const float LDotN = sqrtf( 1.0f - SinThetaT2 );
	const float r1 = (VDotN - eio * LDotN) / (VDotN + eio * LDotN);
	const float r2 = (LDotN - eio * VDotN) / (LDotN + eio * VDotN);
	return 0.5f * (sqrf( r1 ) + sqrf( r2 ));
}
static inline int Refract_L( f3 wi, f3 n, float eta, f3* wt )
{
	const float cosThetaI = fabsf( dot3( n, wi ) );
	const float sin2ThetaI = fmaxf( 0.0f, 1.0f - cosThetaI * cosThetaI );
	const float sin2ThetaT = eta * eta * sin2ThetaI;
	if (sin2ThetaT >= 1) return 0;
	const float cosThetaT = sqrtf( 1.0f - sin2ThetaT );
	*wt = add3( smul( eta, muls( wi, -1.0f ) ), smul( eta * cosThetaI - cosThetaT, n ) );
	return 1;
}
/* ggxmdf.h */
static inline float stretched_roughness( f3 m, float sin_theta, float ax, float ay )
{
	if (ax == ay || sin_theta == 0.0f) return 1.0f / sqrf( ax );
	const float c = sqrf( m.x / (sin_theta * ax) ), s = sqrf( m.y / (sin_theta * ay) );
	return c + s;
}
static inline float projected_roughness( f3 m, float sin_theta, float ax, float ay )
{
	if (ax == ay || sin_theta == 0.0f) return ax;
	const float c = sqrf( (m.x * ax) / sin_theta ), s = sqrf( (m.y * ay) / sin_theta );
	return sqrtf( c + s );
}
static inline float GGXMDF_D( f3 m, float ax, float ay )
{
	const float cos_theta = m.z;
	if (cos_theta == 0.0f) return sqrf( ax ) * INVPI;
	const float cos_theta_2 = sqrf( cos_theta );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	const float cos_theta_4 = sqrf( cos_theta_2 );
	const float tan_theta_2 = (1.0f - cos_theta_2) / cos_theta_2;
	const float A = stretched_roughness( m, sin_theta, ax, ay );
	const float tmp = 1.0f + tan_theta_2 * A;
	return 1.0f / (PI * ax * ay * cos_theta_4 * sqrf( tmp ));
}
static inline float GGXMDF_lambda( f3 v, float ax, float ay )
{
	const float cos_theta = v.z;
	if (cos_theta == 0.0f) return 0.0f;
	const float cos_theta_2 = sqrf( cos_theta );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	const float alpha = projected_roughness( v, sin_theta, ax, ay );
	const float tan_theta_2 = sqrf( sin_theta ) / cos_theta_2;
	const float a2_rcp = sqrf( alpha ) * tan_theta_2;
	return (-1.0f + sqrtf( 1.0f + a2_rcp )) * 0.5f;
}
static inline float GGXMDF_G( f3 wi, f3 wo, float ax, float ay ) { return 1.0f / (1.0f + GGXMDF_lambda( wo, ax, ay ) + GGXMDF_lambda( wi, ax, ay )); }
static inline float GGXMDF_G1( f3 v, float ax, float ay ) { return 1.0f / (1.0f + GGXMDF_lambda( v, ax, ay )); }
static inline f3 GGXMDF_sample( f3 v, float r0, float r1, float ax, float ay )
{
	const float sign_cos_vn = v.z < 0.0f ? -1.0f : 1.0f;
	f3 stretched = mk3( sign_cos_vn * v.x * ax, sign_cos_vn * v.y * ay, sign_cos_vn * v.z );
	stretched = normalize3( stretched );
	const f3 t1 = v.z < 0.9999f ? normalize3( cross3( stretched, mk3( 0, 0, 1 ) ) ) : mk3( 1, 0, 0 );
	const f3 t2 = cross3( t1, stretched );
	const float a = 1.0f / (1.0f + stretched.z);
	const float r = sqrtf( r0 );
	const float phi = r1 < a ? r1 / a * PI : PI + (r1 - a) / (1.0f - a) * PI;
	float sp, cp;
	lh2_sincosf( phi, &sp, &cp );
	const float p1 = r * cp;
	const float p2 = r * sp * (r1 < a ? 1.0f : stretched.z);
	const f3 h = add3( add3( smul( p1, t1 ), smul( p2, t2 ) ), smul( sqrtf( fmaxf( 0.0f, 1.0f - p1 * p1 - p2 * p2 ) ), stretched ) );
	const f3 m = mk3( h.x * ax, h.y * ay, fmaxf( 0.0f, h.z ) );
	return normalize3( m );
}
static inline float GGXMDF_pdf( f3 v, f3 m, float ax, float ay )
{
	const float cos_theta_v = v.z;
	if (cos_theta_v == 0.0f) return 0;
	return GGXMDF_G1( v, ax, ay ) * fabsf( dot3( v, m ) ) * GGXMDF_D( m, ax, ay ) / fabsf( cos_theta_v );
}
static inline float GTR1MDF_D( f3 m, float ax )
{
	const float alpha = clampf_( ax, 0.001f, 0.999f );
	const float alpha_x_2 = sqrf( alpha );
	const float cos_theta_2 = sqrf( m.z );
	const float a = (alpha_x_2 - 1.0f) / (PI * lh2_logf( alpha_x_2 ));
	const float b = (1 / (1 + (alpha_x_2 - 1) * cos_theta_2));
	return a * b;
}
static inline float GTR1MDF_lambda( f3 v, float ax )
{
	const float cos_theta = v.z;
	if (cos_theta == 0) return 0;
	const float cos_theta_2 = sqrf( cos_theta );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	if (sin_theta == 0.0f) return 0.0f;
	const float cot_theta_2 = cos_theta_2 / sqrf( sin_theta );
	const float cot_theta = sqrtf( cot_theta_2 );
	const float alpha = clampf_( ax, 0.001f, 0.999f );
	const float alpha_2 = sqrf( alpha );
	const float a = sqrtf( cot_theta_2 + alpha_2 );
	const float b = sqrtf( cot_theta_2 + 1.0f );
	const float c = lh2_logf( cot_theta + b );
	const float d = lh2_logf( cot_theta + a );
	return (a - b + cot_theta * (c - d)) / (cot_theta * lh2_logf( alpha_2 ));
}
static inline float GTR1MDF_G( f3 wi, f3 wo, float ax ) { return 1.0f / (1.0f + GTR1MDF_lambda( wo, ax ) + GTR1MDF_lambda( wi, ax )); }
static inline f3 GTR1MDF_sample( float r0, float r1, float ax )
{
	const float alpha = clampf_( ax, 0.001f, 0.999f );
	const float alpha_2 = sqrf( alpha );
	const float a = 1.0f - lh2_powf( alpha_2, 1.0f - r0 );
	const float cos_theta_2 = a / (1.0f - alpha_2);
	const float cos_theta = sqrtf( cos_theta_2 );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	float sin_phi, cos_phi;
	lh2_sincosf( TWOPI * r1, &sin_phi, &cos_phi );
	return mk3( cos_phi * sin_theta, sin_phi * sin_theta, cos_theta );
}
static inline float GTR1MDF_pdf( f3 m, float ax ) { return GTR1MDF_D( m, ax ) * fabsf( m.z ); }

#define GGXMDF 1001
#define GTR1MDF 1002
/* disney.h:93-116, flip = false; wiw/pdf/value are left untouched on early exit (see Q1) */
static void sample_mf( int MDF, const ShadingData* sd, float r0, float r1, float ax, float ay,
	f3 N, f3 T, f3 B, f3 gN, f3 wow, f3* wiw, float* pdf, f3* value )
{
	f3 wo = World2Tangent( wow, N, T, B );
	if (wo.z == 0) return;
	f3 m = MDF == GGXMDF ? GGXMDF_sample( wo, r0, r1, ax, ay ) : GTR1MDF_sample( r0, r1, ax );
	f3 wi = reflect3( muls( wo, -1.0f ), m );
	const f3 ng = World2Tangent( gN, N, T, B );
	if (force_above_surface( &wi, ng )) m = normalize3( add3( wo, wi ) );
	if (wi.z == 0) return;
	const float cos_oh = dot3( wo, m );
	*pdf = (MDF == GGXMDF ? GGXMDF_pdf( wo, m, ax, ay ) : GTR1MDF_pdf( m, ax )) / fabsf( 4.0f * cos_oh );
	if (*pdf < 1.0e-6f) return;
	const float D = MDF == GGXMDF ? GGXMDF_D( m, ax, ay ) : GTR1MDF_D( m, ax );
	const float G = MDF == GGXMDF ? GGXMDF_G( wi, wo, ax, ay ) : GTR1MDF_G( wi, wo, ax );
	*value = MDF == GGXMDF ? DisneySpecularFresnel( sd, wo, m ) : DisneyClearcoatFresnel( sd, wo, m );
	*value = muls( *value, D * G / fabsf( 4.0f * wo.z * wi.z ) );
	*wiw = Tangent2World( wi, N, T, B );
}
/* disney.h:118-134; bsdf untouched on early exit */
static float evaluate_mf( int MDF, const ShadingData* sd, float ax, float ay, f3 N, f3 T, f3 B, f3 wow, f3 wiw, f3* bsdf )
{
	const f3 wo = World2Tangent( wow, N, T, B );
	const f3 wi = World2Tangent( wiw, N, T, B );
	if (wo.z == 0 || wi.z == 0) return 0;
	const f3 m = normalize3( add3( wi, wo ) );
	const float cos_oh = dot3( wo, m );
	if (cos_oh == 0) return 0;
	const float D = MDF == GGXMDF ? GGXMDF_D( m, ax, ay ) : GTR1MDF_D( m, ax );
	const float G = MDF == GGXMDF ? GGXMDF_G( wi, wo, ax, ay ) : GTR1MDF_G( wi, wo, ax );
	*bsdf = MDF == GGXMDF ? DisneySpecularFresnel( sd, wo, m ) : DisneyClearcoatFresnel( sd, wo, m );
	*bsdf = muls( *bsdf, D * G / fabsf( 4.0f * wo.z * wi.z ) );
	return (MDF == GGXMDF ? GGXMDF_pdf( wo, m, ax, ay ) : GTR1MDF_pdf( m, ax )) / fabsf( 4.0f * cos_oh );
}
static float evaluate_diffuse( const ShadingData* sd, f3 iN, f3 wow, f3 wiw, f3* value ) /* disney.h:136-164 */
{
	const f3 n = iN;
	const f3 h = normalize3( add3( wiw, wow ) );
	const float cos_on = dot3( n, wow );
	const float cos_in = dot3( n, wiw );
	const float cos_ih = dot3( wiw, h );
	const float fl = schlick_fresnel( cos_in );
	const float fv = schlick_fresnel( cos_on );
	float fd = 0;
	if (SUBSURFACE != 1.0f)
	{
		const float fd90 = 0.5f + 2.0f * sqrf( cos_ih ) * ROUGHNESS;
		fd = mixf( 1.0f, fd90, fl ) * mixf( 1.0f, fd90, fv );
	}
	if (SUBSURFACE > 0)
	{
		const float fss90 = sqrf( cos_ih ) * ROUGHNESS;
		const float fss = mixf( 1.0f, fss90, fl ) * mixf( 1.0f, fss90, fv );
		const float ss = 1.25f * (fss * (1.0f / (fabsf( cos_on ) + fabsf( cos_in )) - 0.5f) + 0.5f);
		fd = mixf( fd, ss, SUBSURFACE );
	}
	*value = muls( muls( muls( sd->color, fd ), INVPI ), 1.0f - METALLIC );
	return fabsf( cos_in ) * INVPI;
}
static float evaluate_sheen( const ShadingData* sd, f3 wow, f3 wiw, f3* value ) /* disney.h:178-187 */
{
	const f3 h = normalize3( add3( wow, wow ) );
	const float cos_ih = dot3( wiw, h );
	const float fh = schlick_fresnel( cos_ih );
	*value = mix_one_with_spectra( TINT, SHEENTINT );
	*value = muls( *value, fh * SHEEN * (1.0f - METALLIC) );
	return 1.0f / (2 * PI);
}
static f3 SampleBSDF( const ShadingData* sd, f3 iN, f3 N, f3 iT, f3 wow, float distance, float r0, float r1,
	f3* wiw, float* pdf, int* specular ) /* disney.h:201-296 */
{
	const float flip = (dot3( wow, N ) < 0) ? -1 : 1;
	iN = muls( iN, flip );
	if (r0 < TRANSMISSION)
	{
		*specular = 1, *pdf = 1;
		const float eio = flip < 0 ? (1.0f / ETA) : ETA, F = Fr_L( dot3( iN, wow ), eio );
		f3 beer;
		beer.x = lh2_expf( -sd->transmittance.x * distance * 2.0f );
		beer.y = lh2_expf( -sd->transmittance.y * distance * 2.0f );
		beer.z = lh2_expf( -sd->transmittance.z * distance * 2.0f );
		if (r1 < F)
		{
			*wiw = reflect3( muls( wow, -1.0f ), iN );
			if (dot3( muls( N, flip ), *wiw ) <= 0) *pdf = 0;
			return muls( mul3( sd->color, beer ), 1 / fabsf( dot3( iN, *wiw ) ) );
		}
		else
		{
			if (!Refract_L( wow, iN, eio, wiw )) return s3( 0 );
			const float ajointCorrection = 1.0f;
			return muls( muls( mul3( sd->color, beer ), ajointCorrection ), 1 / fabsf( dot3( iN, *wiw ) ) );
		}
	}
	const float r3 = (r0 - TRANSMISSION) / (1 - TRANSMISSION);
	const f3 B = normalize3( cross3( iN, iT ) );
	const f3 T = normalize3( cross3( iN, B ) );
	f4 weights = { lerpf_( LUMINANCE, 0, METALLIC ), lerpf_( SHEEN, 0, METALLIC ), lerpf_( SPECULAR, 1, METALLIC ), CLEARCOAT * 0.25f };
	const float wsum = 1.0f / (weights.x + weights.y + weights.z + weights.w);
	weights.x *= wsum, weights.y *= wsum, weights.z *= wsum, weights.w *= wsum;
	const f4 cdf = { weights.x, weights.x + weights.y, weights.x + weights.y + weights.z, 0 };
	float probability, component_pdf = 0; /* Q1 */
	f3 contrib = s3( 0 ), value = s3( 0 );  /* Q1 */
	if (r3 < cdf.x)
	{
		const float r2 = r3 / cdf.x;
		const f3 wi = DiffuseReflectionCosWeighted( r2, r1 );
		*wiw = normalize3( Tangent2World( wi, iN, T, B ) );
		component_pdf = evaluate_diffuse( sd, iN, wow, *wiw, &value );
		probability = weights.x * component_pdf, weights.x = 0;
	}
	else if (r3 < cdf.y)
	{
		const float r2 = (r3 - cdf.x) / (cdf.y - cdf.x);
		const f3 wi = DiffuseReflectionCosWeighted( r2, r1 );
		*wiw = normalize3( Tangent2World( wi, iN, T, B ) );
		component_pdf = evaluate_sheen( sd, wow, *wiw, &value );
		probability = weights.y * component_pdf, weights.y = 0;
	}
	else if (r3 < cdf.z)
	{
		const float r2 = (r3 - cdf.y) / (cdf.z - cdf.y);
		float ax, ay;
		microfacet_alpha_from_roughness( ROUGHNESS, ANISOTROPIC, &ax, &ay );
		sample_mf( GGXMDF, sd, r2, r1, ax, ay, iN, T, B, muls( N, flip ), wow, wiw, &component_pdf, &value );
		probability = weights.z * component_pdf, weights.z = 0;
	}
	else
	{
		const float r2 = (r3 - cdf.z) / (1 - cdf.z);
		const float alpha = clearcoat_roughness( sd );
		sample_mf( GTR1MDF, sd, r2, r1, alpha, alpha, iN, T, B, muls( N, flip ), wow, wiw, &component_pdf, &value );
		probability = weights.w * component_pdf, weights.w = 0;
	}
	if (weights.x > 0) probability += weights.x * evaluate_diffuse( sd, iN, wow, *wiw, &contrib ), value = add3( value, contrib );
	if (weights.y > 0) probability += weights.y * evaluate_sheen( sd, wow, *wiw, &contrib ), value = add3( value, contrib );
	if (weights.z > 0)
	{
		float ax, ay;
		microfacet_alpha_from_roughness( ROUGHNESS, ANISOTROPIC, &ax, &ay );
		probability += weights.z * evaluate_mf( GGXMDF, sd, ax, ay, iN, T, B, wow, *wiw, &contrib );
		value = add3( value, contrib );
	}
	if (weights.w > 0)
	{
		const float alpha = clearcoat_roughness( sd );
		probability += weights.w * evaluate_mf( GTR1MDF, sd, alpha, alpha, iN, T, B, wow, *wiw, &contrib );
		value = add3( value, contrib );
	}
	if (probability > 1.0e-6f) *pdf = probability; else *pdf = 0;
	return value;
}
static f3 EvaluateBSDF( const ShadingData* sd, f3 iN, f3 iT, f3 wow, f3 wiw, float* pdf ) /* disney.h:298-333 */
{
	if (TRANSMISSION > 0.999f || ROUGHNESS <= 0.001f) { *pdf = 0; return s3( 0 ); }
	const f3 B = normalize3( cross3( iN, iT ) );
	const f3 T = normalize3( cross3( iN, B ) );
	f4 weights = { lerpf_( LUMINANCE, 0, METALLIC ), lerpf_( SHEEN, 0, METALLIC ), lerpf_( SPECULAR, 1, METALLIC ), CLEARCOAT * 0.25f };
	const float wsum = 1.0f / (weights.x + weights.y + weights.z + weights.w);
	weights.x *= wsum, weights.y *= wsum, weights.z *= wsum, weights.w *= wsum;
	*pdf = 0;
	f3 value = s3( 0 );
	if (weights.x > 0) *pdf += weights.x * evaluate_diffuse( sd, iN, wow, wiw, &value );
	if (weights.y > 0) *pdf += weights.y * evaluate_sheen( sd, wow, wiw, &value );
	if (weights.z > 0)
	{
		float ax, ay;
		microfacet_alpha_from_roughness( ROUGHNESS, ANISOTROPIC, &ax, &ay );
		f3 contrib = s3( 0 );
		const float spec_pdf = evaluate_mf( GGXMDF, sd, ax, ay, iN, T, B, wow, wiw, &contrib );
		if (spec_pdf > 0) *pdf += weights.z * spec_pdf, value = add3( value, contrib );
	}
	if (weights.w > 0)
	{
		const float alpha = clearcoat_roughness( sd );
		f3 contrib = s3( 0 );
		const float clearcoat_pdf = evaluate_mf( GTR1MDF, sd, alpha, alpha, iN, T, B, wow, wiw, &contrib );
		if (clearcoat_pdf > 0) *pdf += weights.w * clearcoat_pdf, value = add3( value, contrib );
	}
	return value;
}

/* ------------------------------------------------------------------------------------- */
/* camera: kernels/camera.h:22-94                                                          */
/* ------------------------------------------------------------------------------------- */
static f3 RandomPointOnLens( float r0, float r1, f3 pos, float aperture, f3 right, f3 up )
{
	const float blade = (float)(int)(r0 * 9);
	float r2 = (r0 - blade * (1.0f / 9.0f)) * 9.0f;
	float x1, y1, x2, y2;
	lh2_sincosf( blade * PI / 4.5f, &x1, &y1 );
	lh2_sincosf( (blade + 1.0f) * PI / 4.5f, &x2, &y2 );
	if ((r1 + r2) > 1) r1 = 1.0f - r1, r2 = 1.0f - r2;
	const float xr = x1 * r1 + x2 * r2;
	const float yr = y1 * r1 + y2 * r2;
	return add3( pos, smul( aperture, add3( muls( right, xr ), muls( up, yr ) ) ) );
}

typedef struct { f3 O; float tmin; f3 D; float tmax; f4 T4, Q4; } PathSeg;

static void eye_ray( const Oracle* o, const lh2_ViewPyramid* view, uint32_t R0, int pass, int jobIndex, PathSeg* ps )
{
	const int w = o->w, h = o->h;
	const f3 p1 = lf3( view->p1 ), pos = lf3( view->pos );
	const f3 right = sub3( lf3( view->p2 ), p1 ), up = sub3( lf3( view->p3 ), p1 );
	const uint32_t x = (uint32_t)jobIndex % (uint32_t)w;
	uint32_t y = (uint32_t)jobIndex / (uint32_t)w;
	const uint32_t sampleIndex = (uint32_t)pass + y / (uint32_t)h;
	y %= (uint32_t)h;
	float r0, r1, r2, r3;
	if (sampleIndex < 256 && !o->primeRef)   /* PrimeRef camera: uniform random numbers (camera.h:57-59) */
	{
		r0 = blueNoiseSampler( o->blueNoise, x, y, sampleIndex, 0 );
		r1 = blueNoiseSampler( o->blueNoise, x, y, sampleIndex, 1 );
		r2 = blueNoiseSampler( o->blueNoise, x, y, sampleIndex, 2 );
		r3 = blueNoiseSampler( o->blueNoise, x, y, sampleIndex, 3 );
	}
	else
	{
		uint32_t seed = WangHash( (uint32_t)jobIndex + R0 );
		r0 = RandomFloat( &seed ), r1 = RandomFloat( &seed );
		r2 = RandomFloat( &seed ), r3 = RandomFloat( &seed );
	}
	f3 posOnPixel;
	if (view->distortion == 0 || o->primeRef)
	{
		posOnPixel = add3( add3( p1, smul( (float)x + r0, divs( right, (float)w ) ) ), smul( (float)y + r1, divs( up, (float)h ) ) );
	}
	else
	{
		const float sx = (float)x / (float)w - 0.5f, sy = (float)y / (float)h - 0.5f;
		const float rr = sx * sx + sy * sy;
		const float rq = sqrtf( rr ) * (1.0f + view->distortion * rr + view->distortion * rr * rr);
		const float theta = lh2_atan2f( sx, sy );
		float st, ct;
		lh2_sincosf( theta, &st, &ct );
		const float bx = (st * rq + 0.5f) * (float)w;
		const float by = (ct * rq + 0.5f) * (float)h;
		posOnPixel = add3( add3( p1, smul( bx + r0, divs( right, (float)w ) ) ), smul( by + r1, divs( up, (float)h ) ) );
	}
	const f3 posOnLens = RandomPointOnLens( r2, r3, pos, view->aperture, right, up );
	const f3 rayDir = normalize3( sub3( posOnPixel, posOnLens ) );
	ps->O = posOnLens, ps->tmin = o->geometryEpsilon;
	ps->D = rayDir, ps->tmax = 1e34f;
	ps->T4.x = 1, ps->T4.y = 1, ps->T4.z = 1;
	ps->T4.w = bitsf( ((x + (y + (sampleIndex - (uint32_t)pass) * (uint32_t)h) * (uint32_t)w) << 8) + 1 );
	ps->Q4.x = 1, ps->Q4.y = 0, ps->Q4.z = 0, ps->Q4.w = 0;
}

void orc_generate_eye_rays( Oracle* o, const lh2_ViewPyramid* view, uint32_t R0, int pass, float* ot, float* dt, float* st )
{
	const int n = o->w * o->h * o->spp;
	for (int i = 0; i < n; i++)
	{
		PathSeg ps;
		eye_ray( o, view, R0, pass, i, &ps );
		ot[i * 4 + 0] = ps.O.x, ot[i * 4 + 1] = ps.O.y, ot[i * 4 + 2] = ps.O.z, ot[i * 4 + 3] = ps.tmin;
		dt[i * 4 + 0] = ps.D.x, dt[i * 4 + 1] = ps.D.y, dt[i * 4 + 2] = ps.D.z, dt[i * 4 + 3] = ps.tmax;
		memcpy( st + i * 8, &ps.T4, 16 ); memcpy( st + i * 8 + 4, &ps.Q4, 16 );
	}
}

/* ------------------------------------------------------------------------------------- */
/* shade: kernels/pathtracer.h:54-245 (one path vertex); shadow ray traced immediately       */
/* ------------------------------------------------------------------------------------- */
typedef struct { float* acc; OracleStats st; } ThreadCtx;

static inline f3 clampintensity( const Oracle* o, f3 c ) /* core_settings.h:146-148 */
{
	const float v = fmaxf( c.x, fmaxf( c.y, c.z ) );
	if (v > o->clampValue) { const float m = o->clampValue / v; c.x *= m; c.y *= m; c.z *= m; }
	return c;
}
static inline f3 fixnan( f3 a ) { if (!isfinite_( a.x + a.y + a.z )) a = s3( 0 ); return a; } /* common_settings.h:58 */
static inline void acc_add( float* acc, uint32_t px, f3 c, float w )
{
	acc[px * 4 + 0] += c.x, acc[px * 4 + 1] += c.y, acc[px * 4 + 2] += c.z, acc[px * 4 + 3] += w;
}

/* returns 1 and fills *next when an extension ray is produced */
static int shade_one( const Oracle* o, ThreadCtx* ctx, const PathSeg* in, const THit* hd, uint32_t R0, int pass, int pathLength, PathSeg* next )
{
	const int w = o->w, h = o->h;
	const int MAXPL = o->maxPathLength;
	/* hit packing exactly as pathtracer.h:71 */
	const uint32_t uvbits = lh2_f2u( 65535.0f * hd->u ) + (lh2_f2u( 65535.0f * hd->v ) << 16);
	const int PRIMIDX = hd->tri;
	const int INSTANCEIDX = hd->tri == -1 ? 0 : hd->inst;
	const float HIT_U = (float)(uvbits & 65535) * (1.0f / 65535.0f);
	const float HIT_V = (float)(uvbits >> 16) * (1.0f / 65535.0f);
	const float HIT_T = hd->t;
	uint32_t data = fbits( in->T4.w );
	const float bsdfPdf = in->Q4.x;
	const f3 D = in->D;
	f3 throughput = f4xyz( in->T4 );
	const uint32_t pathIdx = data >> 8;
	const uint32_t pixelIdx = pathIdx % (uint32_t)(w * h);
	const uint32_t sampleIdx = pathIdx / (uint32_t)(w * h) + (uint32_t)pass;
	if (pathLength == 1) ctx->acc[pixelIdx * 4 + 3] += PRIMIDX == NOHIT ? 10000 : HIT_T;
	if (PRIMIDX == NOHIT)
	{
		f3 contribution = muls( mul3( throughput, SampleSkydome( o, D ) ), 1.0f / bsdfPdf );
		contribution = clampintensity( o, contribution );
		contribution = fixnan( contribution );
		acc_add( ctx->acc, pixelIdx, contribution, 0 );
		return 0;
	}
	if ((int)pixelIdx == o->probeX + w * o->probeY && pathLength == 1 && sampleIdx == 0)
		ctx->st.probedInstid = INSTANCEIDX, ctx->st.probedTriid = PRIMIDX, ctx->st.probedDist = HIT_T;
	ShadingData sdv, * sd = &sdv;
	f3 N, iN, fN, T;
	const f3 I = add3( in->O, smul( HIT_T, D ) );
	const lh2_CoreTri* tri = &o->meshes[o->inst[INSTANCEIDX].mesh].tris[PRIMIDX];
	GetShadingData( o, D, HIT_U, HIT_V, o->spreadAngle * HIT_T, tri, INSTANCEIDX, sd, &N, &iN, &fN, &T );
	if (sd->flags & 1) /* alpha pass-through (never set without textures) */
	{
		if (pathLength < MAXPL)
		{
			next->O = I, next->tmin = EPSILON, next->D = D, next->tmax = 1e34f;
			throughput = fixnan( throughput );
			next->T4.x = throughput.x, next->T4.y = throughput.y, next->T4.z = throughput.z, next->T4.w = bitsf( data );
			next->Q4.x = bsdfPdf, next->Q4.y = 0, next->Q4.z = 0, next->Q4.w = 0;
			return 1;
		}
		return 0;
	}
	if (sd->color.x > 1.0f || sd->color.y > 1.0f || sd->color.z > 1.0f) /* IsEmissive */
	{
		const float DdotNL = -dot3( D, N );
		f3 contribution = s3( 0 );
		if (DdotNL > 0)
		{
			if (pathLength == 1 || (data & S_SPECULAR) > 0) contribution = sd->color;
			else
			{
				const f3 lastN = UnpackNormal( fbits( in->Q4.y ) );
				const float lightPdf = CalculateLightPDF( D, HIT_T, tri->area, N );
				const float pickProb = LightPickProb( o, tri->ltriIdx, in->O, lastN, I );
				if ((bsdfPdf + lightPdf * pickProb) > 0) contribution = muls( mul3( throughput, sd->color ), 1.0f / (bsdfPdf + lightPdf * pickProb) );
			}
			contribution = clampintensity( o, contribution );
			contribution = fixnan( contribution );
			acc_add( ctx->acc, pixelIdx, contribution, 0 );
		}
		return 0;
	}
	if (ROUGHNESS <= 0.001f || TRANSMISSION > 0.999f) data |= S_SPECULAR; else data &= ~S_SPECULAR;
	uint32_t seed = WangHash( pathIdx * 17 + R0 );
	const float faceDir = (dot3( D, N ) > 0) ? -1 : 1;
	if (faceDir == 1) sd->transmittance = s3( 0 );
	throughput = muls( throughput, 1.0f / bsdfPdf );
	if (!(data & S_SPECULAR))
	{
		float r0, r1, pickProb = 0, lightPdf = 0;
		if (sampleIdx < 2)
		{
			const uint32_t x = (pixelIdx % (uint32_t)w) & 127, y = (pixelIdx / (uint32_t)w) & 127;
			r0 = blueNoiseSampler( o->blueNoise, x, y, sampleIdx, 4 + 4 * pathLength );
			r1 = blueNoiseSampler( o->blueNoise, x, y, sampleIdx, 5 + 4 * pathLength );
		}
		else
		{
			r0 = RandomFloat( &seed );
			r1 = RandomFloat( &seed );
		}
		f3 lightColor = s3( 0 );
		f3 L = sub3( RandomPointOnLight( o, r0, r1, I, muls( fN, faceDir ), &pickProb, &lightPdf, &lightColor ), I );
		const float dist = length3( L );
		L = muls( L, 1.0f / dist );
		const float NdotL = dot3( L, muls( fN, faceDir ) );
		if (NdotL > 0 && lightPdf > 0)
		{
			float bsdfPdf2;
			const f3 sampledBSDF = EvaluateBSDF( sd, fN, T, muls( D, -1.0f ), L, &bsdfPdf2 );
			if (bsdfPdf2 > 0)
			{
				f3 contribution = muls( mul3( mul3( throughput, sampledBSDF ), lightColor ), NdotL / (pickProb * lightPdf + bsdfPdf2) );
				contribution = fixnan( contribution );
				contribution = clampintensity( o, contribution );
				ctx->st.shadowRays++;
				/* fire-and-forget shadow ray (pathtracer.h:202-205) + finalizeConnectionKernel (connections.h:22-34) */
				const f3 SO = SafeOrigin( I, L, muls( N, faceDir ), o->geometryEpsilon );
				THit sh; uint32_t nn = 0, tt = 0; int occluded;
				trace_ray( o, SO, L, 0.0f, dist - 2 * o->geometryEpsilon, 1, &sh, &nn, &tt, &occluded );
				if (!occluded) acc_add( ctx->acc, pixelIdx, contribution, 0 );
				if ((int)pixelIdx == o->debugPixel)
				{
					const float rec[16] = { 1, (float)pathLength, (float)occluded, SO.x, SO.y, SO.z, L.x, L.y, L.z, dist - 2 * o->geometryEpsilon,
						contribution.x, contribution.y, contribution.z, 0, 0, 0 };
					debug_log( o, rec );
				}
			}
		}
	}
	if (data & ENOUGH_BOUNCES || pathLength == MAXPL) return 0;
	f3 R = s3( 0 ); /* Q1 */
	float newBsdfPdf = 0, r3, r4;
	if (sampleIdx < 256)
	{
		const uint32_t x = (pixelIdx % (uint32_t)w) & 127, y = (pixelIdx / (uint32_t)w) & 127;
		r3 = blueNoiseSampler( o->blueNoise, x, y, sampleIdx, 6 + 4 * pathLength );
		r4 = blueNoiseSampler( o->blueNoise, x, y, sampleIdx, 7 + 4 * pathLength );
	}
	else
	{
		r3 = RandomFloat( &seed );
		r4 = RandomFloat( &seed );
	}
	int specular = 0;
	const f3 bsdf = SampleBSDF( sd, fN, N, T, muls( D, -1.0f ), HIT_T, r3, r4, &R, &newBsdfPdf, &specular );
	if (newBsdfPdf < EPSILON || newBsdfPdf != newBsdfPdf) return 0;
	if (specular) data |= S_SPECULAR;
	const float p = ((data & S_SPECULAR) || ((data & S_BOUNCED) == 0)) ? 1 : SurvivalProbability( bsdf );
	if (p < RandomFloat( &seed )) return 0; else throughput = muls( throughput, 1 / p );
	const uint32_t packedNormal = PackNormal( muls( fN, faceDir ) );
	if (!(data & S_SPECULAR)) data |= data & S_BOUNCED ? S_BOUNCEDTWICE : S_BOUNCED; else data |= S_VIASPECULAR;
	next->O = SafeOrigin( I, R, muls( N, faceDir ), o->geometryEpsilon ), next->tmin = 0;
	next->D = R, next->tmax = 1e34f;
	throughput = fixnan( throughput );
	const f3 nt = muls( mul3( throughput, bsdf ), fabsf( dot3( muls( fN, faceDir ), R ) ) );
	next->T4.x = nt.x, next->T4.y = nt.y, next->T4.z = nt.z, next->T4.w = bitsf( data );
	next->Q4.x = newBsdfPdf, next->Q4.y = bitsf( packedNormal ), next->Q4.z = 0, next->Q4.w = 0;
	return 1;
}

/* ------------------------------------------------------------------------------------- */
/* RenderCore::Render (rendercore.cpp:463-609), depth-first per path                       */
/* ------------------------------------------------------------------------------------- */
typedef struct
{
	const Oracle* o; const lh2_ViewPyramid* view; uint32_t camR0; int pass;
	int px0, px1; ThreadCtx ctx;
} RenderJob;


/* ------------------------------------------------------------------------------------- */
/* PrimeRef validation mode: RenderCore_PrimeRef/kernels/pathtracer.h:44-165 + bsdf.h:18-101 */
/* (uniform random numbers, Lambert BSDF, NEE without MIS, Russian roulette every vertex,    */
/* MAXPATHLENGTH 64; the last bounce's shadow rays are never traced; a TIR refraction       */
/* sample leaves the direction (0,0,0); alpha cut-outs are shaded as hits)                 */
/* ------------------------------------------------------------------------------------- */
static inline float FrLambert( float VDotN, float eio )
{
	const float SinThetaT2 = sqrf( eio ) * (1.0f - VDotN * VDotN);
	if (SinThetaT2 > 1.0f) return 1.0f;
	const float LDotN = sqrtf( 1.0f - SinThetaT2 );
	const float r1 = (VDotN - eio * LDotN) / (VDotN + eio * LDotN);
	const float r2 = (LDotN - eio * VDotN) / (LDotN + eio * VDotN);
	return 0.5f * (sqrf( r1 ) + sqrf( r2 ));
}
static inline f3 Tangent2WorldN( f3 V, f3 N )   /* tools_shared.h:211-220 */
{
	const float sign = copysignf( 1.0f, N.z );
	const float a = -1.0f / (sign + N.z);
	const float b = N.x * N.y * a;
	const f3 B = mk3( 1.0f + sign * N.x * N.x * a, sign * b, -sign * N.x );
	const f3 T = mk3( b, sign + N.y * N.y * a, -N.y );
	return add3( add3( smul( V.x, T ), smul( V.y, B ) ), smul( V.z, N ) );
}
static f3 LambertEvaluate( const ShadingData* sd, f3 iN, f3 wi, float* pdf )
{
	if (TRANSMISSION > 0.999f || ROUGHNESS <= 0.001f) { *pdf = 0; return s3( 0 ); }
	*pdf = fabsf( dot3( wi, iN ) ) * INVPI;
	return muls( muls( sd->color, INVPI ), ROUGHNESS );
}
static f3 LambertSample( const ShadingData* sd, f3 iN, f3 N, f3 wo, float distance, float r3, float r4, f3* wi, float* pdf, int* specular )
{
	const float flip = (dot3( wo, N ) < 0) ? -1 : 1;
	iN = muls( iN, flip );
	*specular = 1, *pdf = 1;
	f3 bsdf;
	if (r4 < TRANSMISSION)
	{
		const float eio = flip < 0 ? (1.0f / ETA) : ETA, F = FrLambert( dot3( iN, wo ), eio );
		const f3 beer = mk3( lh2_expf( -sd->transmittance.x * distance * 2.0f ), lh2_expf( -sd->transmittance.y * distance * 2.0f ),
			lh2_expf( -sd->transmittance.z * distance * 2.0f ) );
		if (r3 < F)
		{
			*wi = reflect3( muls( wo, -1.0f ), iN );
			bsdf = muls( mul3( sd->color, beer ), 1 / fabsf( dot3( iN, *wi ) ) );
		}
		else
		{
			if (!Refract_L( wo, iN, eio, wi )) return s3( 0 );
			return muls( mul3( sd->color, beer ), 1 / fabsf( dot3( iN, *wi ) ) );
		}
	}
	else
	{
		const float pReflect = 1 - ROUGHNESS;
		if (r3 < pReflect)
		{
			*wi = reflect3( muls( wo, -1.0f ), iN );
			bsdf = muls( sd->color, 1.0f / fabsf( dot3( iN, *wi ) ) );
		}
		else
		{
			const float r5 = (r3 - pReflect) / (1 - pReflect);
			const float r6 = (r4 - TRANSMISSION) / (1 - TRANSMISSION);
			*wi = normalize3( Tangent2WorldN( DiffuseReflectionCosWeighted( r5, r6 ), iN ) );
			*pdf = fmaxf( 0.0f, dot3( *wi, iN ) ) * INVPI;
			*specular = 0;
			bsdf = muls( sd->color, INVPI );
		}
	}
	if (dot3( muls( N, flip ), *wi ) <= 0) *pdf = 0;
	return bsdf;
}
static int shade_one_ref( const Oracle* o, ThreadCtx* ctx, const PathSeg* in, const THit* hd, uint32_t R0, int pass, int pathLength, int MAXPL, PathSeg* next )
{
	const int w = o->w, h = o->h;
	const uint32_t uvbits = lh2_f2u( 65535.0f * hd->u ) + (lh2_f2u( 65535.0f * hd->v ) << 16);
	const int PRIMIDX = hd->tri;
	const int INSTANCEIDX = hd->tri == -1 ? 0 : hd->inst;
	const float HIT_U = (float)(uvbits & 65535) * (1.0f / 65535.0f);
	const float HIT_V = (float)(uvbits >> 16) * (1.0f / 65535.0f);
	const float HIT_T = hd->t;
	uint32_t data = fbits( in->T4.w );
	const f3 D = in->D;
	f3 throughput = f4xyz( in->T4 );
	const uint32_t pathIdx = data >> 8;
	const uint32_t pixelIdx = pathIdx % (uint32_t)(w * h);
	const uint32_t sampleIdx = pathIdx / (uint32_t)(w * h) + (uint32_t)pass;
	if (pathLength == 1) ctx->acc[pixelIdx * 4 + 3] += PRIMIDX == NOHIT ? 10000 : HIT_T;
	if (PRIMIDX == NOHIT)
	{
		acc_add( ctx->acc, pixelIdx, mul3( throughput, SampleSkydome( o, D ) ), 0 );
		return 0;
	}
	if ((int)pixelIdx == o->probeX + w * o->probeY && pathLength == 1 && sampleIdx == 0)
		ctx->st.probedInstid = INSTANCEIDX, ctx->st.probedTriid = PRIMIDX, ctx->st.probedDist = HIT_T;
	ShadingData sdv, * sd = &sdv;
	f3 N, iN, fN, T;
	const f3 I = add3( in->O, smul( HIT_T, D ) );
	const lh2_CoreTri* tri = &o->meshes[o->inst[INSTANCEIDX].mesh].tris[PRIMIDX];
	GetShadingData( o, D, HIT_U, HIT_V, o->spreadAngle * HIT_T, tri, INSTANCEIDX, sd, &N, &iN, &fN, &T );
	if (sd->color.x > 1.0f || sd->color.y > 1.0f || sd->color.z > 1.0f)
	{
		if (-dot3( D, N ) > 0 && (pathLength == 1 || (data & S_SPECULAR))) acc_add( ctx->acc, pixelIdx, mul3( throughput, sd->color ), 0 );
		return 0;
	}
	if (ROUGHNESS <= 0.001f || TRANSMISSION > 0.999f) data |= S_SPECULAR; else data &= ~S_SPECULAR;
	uint32_t seed = WangHash( pathIdx * 17 + R0 );
	const float faceDir = (dot3( D, N ) > 0) ? -1 : 1;
	if (faceDir == 1) sd->transmittance = s3( 0 );
	if (!(data & S_SPECULAR))
	{
		const float r0 = RandomFloat( &seed ), r1 = RandomFloat( &seed );
		float pickProb = 0, lightPdf = 0;
		f3 lightColor = s3( 0 );
		f3 L = sub3( RandomPointOnLight( o, r0, r1, I, muls( fN, faceDir ), &pickProb, &lightPdf, &lightColor ), I );
		const float dist = length3( L );
		L = muls( L, 1.0f / dist );
		const float NdotL = dot3( L, muls( fN, faceDir ) );
		if (NdotL > 0 && lightPdf > 0 && pathLength < MAXPL)
		{
			float bsdfPdf;
			const f3 sampledBSDF = LambertEvaluate( sd, fN, L, &bsdfPdf );
			const f3 contribution = muls( mul3( mul3( throughput, sampledBSDF ), lightColor ), NdotL / (pickProb * lightPdf) );
			ctx->st.shadowRays++;
			const f3 SO = SafeOrigin( I, L, muls( N, faceDir ), o->geometryEpsilon );
			THit sh; uint32_t nn = 0, tt = 0; int occluded;
			trace_ray( o, SO, L, 0.0f, dist - 2 * o->geometryEpsilon, 1, &sh, &nn, &tt, &occluded );
			if (!occluded) acc_add( ctx->acc, pixelIdx, contribution, 0 );
		}
	}
	const float r3 = RandomFloat( &seed ), r4 = RandomFloat( &seed ), r5 = RandomFloat( &seed );
	f3 R = s3( 0 );
	float newBsdfPdf = 0;
	int specular = 0;
	const f3 bsdf = LambertSample( sd, fN, N, muls( D, -1.0f ), HIT_T, r3, r4, &R, &newBsdfPdf, &specular );
	if (newBsdfPdf < EPSILON || newBsdfPdf != newBsdfPdf) return 0;
	if (specular) data |= S_SPECULAR;
	const float p = pathLength == MAXPL ? 0 : ((data & S_SPECULAR) ? 1 : SurvivalProbability( bsdf ));
	if (p <= r5) return 0;
	throughput = mul3( throughput, divs( muls( bsdf, fabsf( dot3( fN, R ) ) ), p * newBsdfPdf ) );
	next->O = SafeOrigin( I, R, muls( N, faceDir ), o->geometryEpsilon ), next->tmin = 0;
	next->D = R, next->tmax = 1e34f;
	next->T4.x = throughput.x, next->T4.y = throughput.y, next->T4.z = throughput.z, next->T4.w = bitsf( data );
	next->Q4.x = 1, next->Q4.y = 0, next->Q4.z = 0, next->Q4.w = 0;
	return 1;
}

static void* render_worker( void* arg )
{
	RenderJob* j = (RenderJob*)arg;
	const Oracle* o = j->o;
	const int np = o->w * o->h;
	for (int s = 0; s < o->spp; s++) for (int px = j->px0; px < j->px1; px++)
	{
		if (o->band > 0 && ((px / o->w) / o->band) % o->bandCount != o->bandRank) continue;
		const int jobIndex = px + s * np;
		PathSeg cur, nxt;
		eye_ray( o, j->view, j->camR0, j->pass, jobIndex, &cur );
		const int MAXPL = o->primeRef ? 64 : o->maxPathLength;   /* PrimeRef: MAXPATHLENGTH 64 */
		for (int pathLength = 1; pathLength <= MAXPL; pathLength++)
		{
			THit hit; uint32_t nn = 0, tt = 0; int occ;
			trace_ray( o, cur.O, cur.D, cur.tmin, cur.tmax, 0, &hit, &nn, &tt, &occ );
			if (hit.tri == -1) hit.t = -1.0f, hit.inst = -1;
			if (px == o->debugPixel)
			{
				float rec[16] = { 0, (float)pathLength, hit.t, 0, 0, cur.O.x, cur.O.y, cur.O.z, cur.D.x, cur.D.y, cur.D.z, cur.tmin, cur.tmax, 0, 0, 0 };
				memcpy( &rec[3], &hit.tri, 4 ), memcpy( &rec[4], &hit.inst, 4 );
				debug_log( o, rec );
			}
			if (pathLength <= 16) j->ctx.st.rayCount[pathLength - 1]++;
			if (pathLength > (int)j->ctx.st.maxPathLength) j->ctx.st.maxPathLength = pathLength;
			const uint32_t R0 = (uint32_t)j->pass * 7907u + (uint32_t)pathLength * 91771u;
			if (o->primeRef ? !shade_one_ref( o, &j->ctx, &cur, &hit, R0, j->pass, pathLength, MAXPL, &nxt )
				: !shade_one( o, &j->ctx, &cur, &hit, R0, j->pass, pathLength, &nxt )) break;
			cur = nxt;
		}
	}
	return 0;
}

void orc_render( Oracle* o, const lh2_ViewPyramid* view, int converge, int nthreads )
{
	if (converge == LH2_RESTART || o->firstConvergingFrame)
	{
		memset( o->acc, 0, sizeof( float ) * 4 * o->w * o->h );
		o->samplesTaken = 0;
		o->firstConvergingFrame = 1;
		o->camRNGseed = 0x12345678;
	}
	if (converge == LH2_CONVERGE) o->firstConvergingFrame = 0;
	o->spreadAngle = view->spreadAngle;
	const uint32_t camR0 = RandomInt( &o->camRNGseed );
	if (nthreads < 1) nthreads = 1;
	const int np = o->w * o->h;
	const int ty0 = o->tileY0 < 0 ? 0 : o->tileY0, ty1 = (o->tileY1 < 0 || o->tileY1 > o->h) ? o->h : o->tileY1;
	const int p0 = ty0 * o->w, p1 = ty1 > ty0 ? ty1 * o->w : p0;
	if (nthreads > p1 - p0) nthreads = p1 - p0 > 0 ? p1 - p0 : 1;
	RenderJob* jobs = (RenderJob*)calloc( nthreads, sizeof( RenderJob ) );
	pthread_t* th = (pthread_t*)calloc( nthreads, sizeof( pthread_t ) );
	for (int t = 0; t < nthreads; t++)
	{
		jobs[t].o = o, jobs[t].view = view, jobs[t].camR0 = camR0, jobs[t].pass = o->samplesTaken;
		jobs[t].px0 = p0 + (int)((long long)(p1 - p0) * t / nthreads), jobs[t].px1 = p0 + (int)((long long)(p1 - p0) * (t + 1) / nthreads);
		jobs[t].ctx.acc = (float*)calloc( (size_t)np * 4, sizeof( float ) );
		jobs[t].ctx.st.probedInstid = jobs[t].ctx.st.probedTriid = -1;
		if (nthreads > 1) pthread_create( &th[t], 0, render_worker, &jobs[t] ); else render_worker( &jobs[t] );
	}
	memset( &o->stats, 0, sizeof( OracleStats ) );
	o->stats.probedInstid = o->stats.probedTriid = -1;
	for (int t = 0; t < nthreads; t++)
	{
		if (nthreads > 1) pthread_join( th[t], 0 );
		/* each thread owns a disjoint pixel range: add its partial accumulator */
		for (int px = jobs[t].px0; px < jobs[t].px1; px++) for (int c = 0; c < 4; c++) o->acc[px * 4 + c] += jobs[t].ctx.acc[px * 4 + c];
		for (int i = 0; i < 16; i++) o->stats.rayCount[i] += jobs[t].ctx.st.rayCount[i];
		o->stats.shadowRays += jobs[t].ctx.st.shadowRays;
		if (jobs[t].ctx.st.maxPathLength > o->stats.maxPathLength) o->stats.maxPathLength = jobs[t].ctx.st.maxPathLength;
		if (jobs[t].ctx.st.probedTriid != -1)
			o->stats.probedInstid = jobs[t].ctx.st.probedInstid, o->stats.probedTriid = jobs[t].ctx.st.probedTriid, o->stats.probedDist = jobs[t].ctx.st.probedDist;
		free( jobs[t].ctx.acc );
	}
	free( jobs ); free( th );
	o->samplesTaken += o->spp;
}

void orc_get_accumulator( const Oracle* o, float* out4 ) { memcpy( out4, o->acc, sizeof( float ) * 4 * o->w * o->h ); }
int orc_samples_taken( const Oracle* o ) { return o->samplesTaken; }
void orc_get_stats( const Oracle* o, OracleStats* s ) { *s = o->stats; }

/* ------------------------------------------------------------------------------------- */
/* unit-level traversal entry points                                                       */
/* ------------------------------------------------------------------------------------- */
typedef struct { const Oracle* o; const float* ot; const float* dt; int i0, i1; uint32_t* hits; uint32_t* visits; } TraceJob;
static void* trace_worker( void* arg )
{
	TraceJob* j = (TraceJob*)arg;
	for (int i = j->i0; i < j->i1; i++)
	{
		THit hit; uint32_t nn = 0, tt = 0; int occ;
		trace_ray( j->o, mk3( j->ot[i * 4], j->ot[i * 4 + 1], j->ot[i * 4 + 2] ), mk3( j->dt[i * 4], j->dt[i * 4 + 1], j->dt[i * 4 + 2] ),
			j->ot[i * 4 + 3], j->dt[i * 4 + 3], 0, &hit, &nn, &tt, &occ );
		if (hit.tri == -1) { j->hits[i * 4 + 0] = fbits( -1.0f ); j->hits[i * 4 + 1] = 0xffffffffu; j->hits[i * 4 + 2] = 0xffffffffu; j->hits[i * 4 + 3] = 0; }
		else
		{
			j->hits[i * 4 + 0] = fbits( hit.t );
			j->hits[i * 4 + 1] = (uint32_t)hit.tri;
			j->hits[i * 4 + 2] = (uint32_t)hit.inst;
			j->hits[i * 4 + 3] = lh2_f2u( 65535.0f * hit.u ) + (lh2_f2u( 65535.0f * hit.v ) << 16);
		}
		if (j->visits) j->visits[i * 2] = nn, j->visits[i * 2 + 1] = tt;
	}
	return 0;
}
void orc_trace_closest( const Oracle* o, const float* ot, const float* dt, int n, uint32_t* hits, uint32_t* visits, int nthreads )
{
	if (nthreads < 1) nthreads = 1;
	if (nthreads > n) nthreads = n > 0 ? n : 1;
	TraceJob* jobs = (TraceJob*)calloc( nthreads, sizeof( TraceJob ) );
	pthread_t* th = (pthread_t*)calloc( nthreads, sizeof( pthread_t ) );
	for (int t = 0; t < nthreads; t++)
	{
		jobs[t].o = o, jobs[t].ot = ot, jobs[t].dt = dt, jobs[t].hits = hits, jobs[t].visits = visits;
		jobs[t].i0 = (int)((long long)n * t / nthreads), jobs[t].i1 = (int)((long long)n * (t + 1) / nthreads);
		if (nthreads > 1) pthread_create( &th[t], 0, trace_worker, &jobs[t] ); else trace_worker( &jobs[t] );
	}
	if (nthreads > 1) for (int t = 0; t < nthreads; t++) pthread_join( th[t], 0 );
	free( jobs ); free( th );
}
void orc_trace_any( const Oracle* o, const float* ot, const float* dt, int n, uint32_t* occl )
{
	memset( occl, 0, sizeof( uint32_t ) * ((n + 31) / 32) );
	for (int i = 0; i < n; i++)
	{
		THit hit; uint32_t nn = 0, tt = 0; int occ;
		trace_ray( o, mk3( ot[i * 4], ot[i * 4 + 1], ot[i * 4 + 2] ), mk3( dt[i * 4], dt[i * 4 + 1], dt[i * 4 + 2] ), ot[i * 4 + 3], dt[i * 4 + 3], 1, &hit, &nn, &tt, &occ );
		if (occ) occl[i >> 5] |= 1u << (i & 31);
	}
}

/* ------------------------------------------------------------------------------------- */
/* KATs                                                                                    */
/* ------------------------------------------------------------------------------------- */
uint32_t orc_wanghash( uint32_t s ) { return WangHash( s ); }
uint32_t orc_xorshift( uint32_t s ) { return RandomInt( &s ); }
float orc_bluenoise( const Oracle* o, int x, int y, int si, int dim ) { return blueNoiseSampler( o->blueNoise, x, y, si, dim ); }
uint32_t orc_pack_normal( float x, float y, float z ) { return PackNormal( mk3( x, y, z ) ); }
void orc_unpack_normal( uint32_t p, float* out ) { const f3 n = UnpackNormal( p ); out[0] = n.x, out[1] = n.y, out[2] = n.z; }

void orc_set_tile( Oracle* o, int y0, int y1 ) { o->tileY0 = y0, o->tileY1 = y1, o->band = 0; }
void orc_set_tile_bands( Oracle* o, int rank, int nranks, int band ) { o->tileY0 = 0, o->tileY1 = -1, o->bandRank = rank, o->bandCount = nranks, o->band = band; }

/* elementary-function evaluation for tests/test_detmath.py */
void orc_detmath_eval( int fn, const float* x, const float* y, int n, float* out )
{
	for (int i = 0; i < n; i++)
	{
		switch (fn)
		{
		case 0: out[i] = lh2_sinf( x[i] ); break;
		case 1: out[i] = lh2_cosf( x[i] ); break;
		case 2: out[i] = lh2_expf( x[i] ); break;
		case 3: out[i] = lh2_logf( x[i] ); break;
		case 4: out[i] = lh2_powf( x[i], y[i] ); break;
		case 5: out[i] = lh2_atan2f( x[i], y[i] ); break;
		case 6: out[i] = lh2_acosf( x[i] ); break;
		case 7: out[i] = lh2_h2f( lh2_f2h( x[i] ) ); break;
		case 8: out[i] = (float)lh2_f2u( x[i] ); break;
		default: out[i] = 0;
		}
	}
}
