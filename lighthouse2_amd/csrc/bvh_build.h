/* bvh_build.h - binned-SAH BVH2 builder producing the GPU child-pair node layout.

   Algorithm family: RenderCore_Bart/bvh.cpp:57-256 (binned SAH, surface-area x count cost, leaves
   for small or unsplittable ranges).  MI355X-first changes: O(N) per level via a bin sweep
   (Bart re-partitions per candidate plane), 16 bins, traversal/intersection cost model, leaves
   capped at 8 primitives, parallel subtrees, and an output layout in which each 64-B node holds
   both children's boxes (lh2_device.h).  Hit results do not depend on the tree (tie rule
   (t, instance, triangle)), only the traversal cost does.
*/
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <vector>

namespace lh2 {

struct Aabb { float lo[3], hi[3]; };

struct BvhOutput
{
	std::vector<float> nodes;      /* 16 floats per node (child-pair layout), node 0 = root */
	std::vector<uint32_t> perm;    /* leaf order -> primitive index */
	int maxDepth = 0;              /* interior levels on the deepest root-to-leaf path */
	int leafCount = 0;
	double sah = 0;                /* SAH cost of the tree (diagnostics) */
};

/* prims: per-primitive bounds; maxLeaf: largest leaf; threads: worker threads (0 = hw);
   traversalCost: SAH cost of a node visit relative to one triangle test; sweepMax: nodes of at most
   this many primitives split by an exact SAH sweep over the sorted centroids (0: binned only);
   triVerts (9 floats per primitive: the triangle's vertices), spatialAlpha > 0 and spatialBudget > 0:
   spatial splits (SBVH) where the object split's children overlap by more than spatialAlpha x the
   root's surface area, adding at most spatialBudget x N references (out.perm then repeats primitives);
   spatialMinRefs: nodes of fewer references try the object split only */
void BuildBvh2( const std::vector<Aabb>& prims, int maxLeaf, int threads, BvhOutput& out, float traversalCost = 1.0f, int sweepMax = 0,
	const float* triVerts = nullptr, float spatialAlpha = 0.0f, float spatialBudget = 0.0f, int spatialMinRefs = 0 );

/* BVH2 (16 floats per node, root 0) -> BVH4 (32 floats per node, root 0; layout: lh2_device.h) by
   greedy surface-area collapse; returns the BVH4 depth (interior levels) */
int CollapseBvh4( const float* nodes2, size_t nodeCount2, std::vector<float>& nodes4 );

/* the same by dynamic programming over surface-area costs (node step 1, leaf visit cLeaf + cTri per
   triangle); subtrees of at most maxLeafTris triangles may become one leaf (BVH2 leaves in DFS order) */
int CollapseBvh4Sah( const float* nodes2, size_t nodeCount2, std::vector<float>& nodes4, float cLeaf, float cTri, int maxLeafTris );


}  // namespace lh2
