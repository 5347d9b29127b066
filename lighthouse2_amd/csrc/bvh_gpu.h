/* bvh_gpu.h - GPU construction of the BVH2 the traversal kernels read (SURVEY.md §8f row 1:
   "GPU BLAS build + per-frame TLAS", replacing the OptiX Prime model builds of
   RenderCore_OptixPrime_B/core_mesh.cpp:36-67 (BLAS) and rendercore.cpp:250-270 (TLAS)).

   Algorithm: PLOC, parallel locally-ordered clustering (Meister & Bittner 2018): primitives sorted
   by 63-bit Morton code of their centroid, then rounds of (nearest neighbour within a window of
   +-radius clusters by merged-box surface area) -> (merge mutual nearest neighbours) -> (compact).
   Ties are broken on (area, lower index, higher index), one total order, so every round merges at
   least one pair.  A node's SAH cost is known when it is created (its children are older), so the
   leaf collapse (subtree of <= maxLeaf primitives kept as one leaf when that is cheaper) happens in
   the same pass.  The output is written by a walk-up pass: each node sums, over its path to the
   root, the interior nodes and primitives of the left siblings, which gives its depth-first
   pre-order slot and its first primitive; so the emitted layout is the one bvh_build.cpp emits
   (child-pair 64-B nodes in DFS pre-order, leaf-ordered 48-B triangles; lh2_device.h).

   Hit results do not depend on the tree (the closest hit is unique under the (t, instance,
   triangle) tie rule and box tests only cull), so the parity tests hold for either builder.
   TLAS builds of up to LH2_TLAS_WG_MAX instances run as one workgroup entirely on the device
   (no host round trip per frame); larger ones and BLAS builds run as a kernel sequence.
*/
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LH2_TLAS_WG_MAX 4096

namespace lh2 {

struct GpuBuildResult
{
	int nodeCount = 0;   /* emitted child-pair nodes */
	int maxDepth = 0;    /* interior levels on the deepest root-to-leaf path (root = 1) */
	int rounds = 0;      /* PLOC rounds */
	float lo[3], hi[3];  /* bounds of all primitives */
};

struct GpuTlasArgs
{
	const float* T;              /* device: 16 floats (row-major 4x4) per instance */
	const int* instMesh;         /* device: mesh index per instance */
	const float* meshBounds;     /* device: 6 floats (lo, hi) per mesh; lo.x > hi.x = empty mesh */
	int count;                   /* instances (>= 2) */
	int nodeBase;                /* index of the TLAS root in the node array */
	float4* nodes;               /* node array; the TLAS is written at nodeBase (<= count - 1 nodes) */
	int maxBlasDepth;            /* stack check: tlasFactor x TLAS depth + this must stay below LH2_STACK_TOTAL - 1 */
	int tlasFactor = 1;          /* stack entries per TLAS level */
	int* sceneError;             /* device flag: set when the stack check fails (traversal then exits) */
	int* tlasDepth;              /* device: TLAS depth out */
};

class GpuBvhBuilder
{
public:
	GpuBvhBuilder() = default;
	GpuBvhBuilder( const GpuBvhBuilder& ) = delete;
	GpuBvhBuilder& operator=( const GpuBvhBuilder& ) = delete;
	~GpuBvhBuilder();

	int radius = 16;   /* PLOC search window (clusters on each side), 1..32 */

	/* BLAS over the CoreTri records already on the device (11 float4 per triangle, vertex0..2 at
	   float4 8..10).  Allocates *nodesOut (4 float4 per node, local refs) and *trisOut (3 float4 per
	   triangle) with hipMalloc; the caller frees them.  triCount >= 2.  Synchronous. */
	void BuildBlas( const float4* coreTris, int triCount, int maxLeaf, float traversalCost, float4** nodesOut, float4** trisOut,
		GpuBuildResult& res, hipStream_t stream );
	/* TLAS over instance world bounds, one instance per leaf, written straight into the node array.
	   Asynchronous for count <= LH2_TLAS_WG_MAX, otherwise synchronous. */
	void BuildTlas( const GpuTlasArgs& a, hipStream_t stream );
	/* copy a mesh's nodes into the scene node array, offsetting interior refs by nodeBase and
	   leaf triangle indices by triBase (asynchronous) */
	static void Relocate( const float4* src, int nodeCount, int nodeBase, uint32_t triBase, float4* dst, hipStream_t stream );
	/* the same for BVH4 nodes (128 B) */
	static void Relocate4( const float4* src, int nodeCount, int nodeBase, uint32_t triBase, float4* dst, hipStream_t stream );
	/* TLAS BVH2 nodes [base2, base2 + count) as two-child BVH4 nodes at base4 (interior refs remapped) */
	static void TlasToBvh4( const float4* nodes2, int base2, int count, int base4, float4* nodes4, hipStream_t stream );
	/* BVH4 nodes [first, first + count) with quantized child boxes (4 uint4 per node, lh2_box4.inc box4q):
	   8-bit child planes on a per-node, per-axis power-of-two grid, rounded outward; a node beyond the grid's range
	   sets LH2_SCENE_ERR_QRANGE in *sceneError */
	static void Quantize4( const float4* nodes4, int first, int count, uint4* q, int* sceneError, hipStream_t stream );

private:
	void Reserve( int n, hipStream_t stream );
	void Cluster( int N, int maxLeaf, float traversalCost, int tlas, GpuBuildResult& res, hipStream_t stream );
	void* Scratch( size_t bytes, hipStream_t stream );

	int cap = 0;
	void* boxes = nullptr;      /* Box8[2 cap]: node boxes */
	void* prim = nullptr;       /* Box8[cap]: primitive boxes (input order) */
	void* cl[2] = {};           /* Box8[cap] cluster boxes, double-buffered */
	int* clNode[2] = {};
	int* child = nullptr;       /* int2[2 cap] */
	int* parent = nullptr;      /* [2 cap] */
	uint32_t* P = nullptr;      /* primitives in subtree */
	uint32_t* I = nullptr;      /* emitted interior nodes in subtree (0: leaf / collapsed) */
	float* cost = nullptr;
	uint32_t* leafOrig = nullptr;
	int* nn = nullptr;
	uint64_t* keys[2] = {};
	uint32_t* vals[2] = {};
	uint64_t* flags = nullptr;
	uint64_t* scan = nullptr;
	uint32_t* dred = nullptr;   /* 16 words: bounds reduction + counters */
	uint32_t* hred = nullptr;   /* pinned mirror */
	void* tmp = nullptr;
	size_t tmpBytes = 0;
	hipStream_t lastStream = nullptr;   /* the stream of the last build (its uses of the scratch end there) */
	hipStream_t retireStream = nullptr; /* ... and of the build before the current one (Reserve) */
};

}  // namespace lh2
