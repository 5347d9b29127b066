/* bvh_build.cpp - parallel binned-SAH BVH2 builder (see bvh_build.h). */
#include "bvh_build.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <thread>

namespace lh2 {

namespace {

#ifndef LH2_SAH_BINS
#define LH2_SAH_BINS 32   /* A/B 8/16/32/64 bins: 32 best by 1-3 % (profiles/r01b_ab_sah_bins.jsonl) */
#endif
constexpr int BINS = LH2_SAH_BINS;
/* build-time A/B knobs of the spatial splits (profiles/r04d_sbvh_build.txt): fewer spatial bins, the object split's axis
   only, or no spatial split below a node size each cut the build time by a third to a half but cost config-2 traversal
   3-6 % more node steps per ray (0.3 % at a minimum of 64 references); the defaults keep the full search */
#ifndef LH2_SBVH_BINS
#define LH2_SBVH_BINS 32
#endif
#ifndef LH2_SBVH_AXES
#define LH2_SBVH_AXES 0
#endif
constexpr int SBINS = LH2_SBVH_BINS;
constexpr float C_ISECT = 1.0f;   /* node-visit cost C_TRAV is a build parameter (relative to one triangle test) */
constexpr uint32_t PAR_THRESHOLD = 16384;

struct TNode { Aabb box; int left, right; uint32_t first, count; };

inline void grow( Aabb& a, const Aabb& b )
{
	for (int k = 0; k < 3; k++) a.lo[k] = std::min( a.lo[k], b.lo[k] ), a.hi[k] = std::max( a.hi[k], b.hi[k] );
}
inline Aabb empty_box()
{
	Aabb a;
	for (int k = 0; k < 3; k++) a.lo[k] = std::numeric_limits<float>::max(), a.hi[k] = -std::numeric_limits<float>::max();
	return a;
}
inline float area( const Aabb& a )
{
	const float dx = a.hi[0] - a.lo[0], dy = a.hi[1] - a.lo[1], dz = a.hi[2] - a.lo[2];
	if (dx < 0 || dy < 0 || dz < 0) return 0;
	return 2.0f * (dx * dy + dx * dz + dy * dz);
}

struct Builder
{
	const std::vector<Aabb>& prims;
	std::vector<float> cent;      /* 3 per prim */
	std::vector<uint32_t> idx;
	std::vector<TNode> nodes;
	std::atomic<int> nodeCount{ 0 };
	std::atomic<int> threadsLeft{ 0 };
	int maxLeaf;
	float C_TRAV = 1.0f;
	uint32_t sweepMax = 0;        /* nodes of at most this many primitives: exact SAH sweep over sorted centroids */

	explicit Builder( const std::vector<Aabb>& p ) : prims( p ) {}

	int alloc2() { return nodeCount.fetch_add( 2 ); }

	void make_leaf( int ni, uint32_t first, uint32_t count, const Aabb& box )
	{
		TNode& n = nodes[ni];
		n.box = box, n.left = n.right = -1, n.first = first, n.count = count;
	}

	void build( int ni, uint32_t first, uint32_t count )
	{
		Aabb box = empty_box(), cbox = empty_box();
		for (uint32_t i = first; i < first + count; i++)
		{
			const uint32_t p = idx[i];
			grow( box, prims[p] );
			for (int k = 0; k < 3; k++) cbox.lo[k] = std::min( cbox.lo[k], cent[p * 3 + k] ), cbox.hi[k] = std::max( cbox.hi[k], cent[p * 3 + k] );
		}
		if (count <= (uint32_t)std::min( 2, maxLeaf )) { make_leaf( ni, first, count, box ); return; }
		/* binned SAH over the three axes */
		float bestCost = std::numeric_limits<float>::max();
		int bestAxis = -1, bestBin = -1;
		const float parentArea = area( box );
		for (int a = 0; a < 3; a++)
		{
			const float ext = cbox.hi[a] - cbox.lo[a];
			if (!(ext > 0)) continue;
			const float scale = (float)BINS * 0.99999f / ext;
			Aabb bb[BINS]; uint32_t bc[BINS];
			for (int b = 0; b < BINS; b++) bb[b] = empty_box(), bc[b] = 0;
			for (uint32_t i = first; i < first + count; i++)
			{
				const uint32_t p = idx[i];
				int b = (int)((cent[p * 3 + a] - cbox.lo[a]) * scale);
				b = std::min( std::max( b, 0 ), BINS - 1 );
				bc[b]++, grow( bb[b], prims[p] );
			}
			float rightArea[BINS]; uint32_t rightCount[BINS];
			Aabb acc = empty_box(); uint32_t n = 0;
			for (int b = BINS - 1; b > 0; b--) { grow( acc, bb[b] ); n += bc[b]; rightArea[b] = area( acc ), rightCount[b] = n; }
			acc = empty_box(); n = 0;
			for (int b = 0; b < BINS - 1; b++)
			{
				grow( acc, bb[b] ); n += bc[b];
				if (n == 0 || rightCount[b + 1] == 0) continue;
				const float cost = C_TRAV + C_ISECT * (area( acc ) * n + rightArea[b + 1] * rightCount[b + 1]) / std::max( parentArea, 1e-30f );
				if (cost < bestCost) bestCost = cost, bestAxis = a, bestBin = b;
			}
		}
		/* exact SAH sweep for small nodes: every split position of the centroid order on each axis */
		uint32_t sweepMid = 0;
		if (count <= sweepMax)
		{
			std::vector<uint32_t> order( count ), bestOrder;
			std::vector<float> rightArea( count + 1 );
			for (int a = 0; a < 3; a++)
			{
				std::copy( idx.begin() + first, idx.begin() + first + count, order.begin() );
				std::sort( order.begin(), order.end(), [&]( uint32_t p, uint32_t q ) { return cent[p * 3 + a] < cent[q * 3 + a] || (cent[p * 3 + a] == cent[q * 3 + a] && p < q); } );
				Aabb acc = empty_box();
				for (uint32_t i = count; i-- > 1;) { grow( acc, prims[order[i]] ); rightArea[i] = area( acc ); }
				acc = empty_box();
				for (uint32_t i = 1; i < count; i++)
				{
					grow( acc, prims[order[i - 1]] );
					const float cost = C_TRAV + C_ISECT * (area( acc ) * (float)i + rightArea[i] * (float)(count - i)) / std::max( parentArea, 1e-30f );
					if (cost < bestCost) bestCost = cost, bestAxis = a, sweepMid = i, bestOrder = order;
				}
			}
			if (sweepMid) std::copy( bestOrder.begin(), bestOrder.end(), idx.begin() + first );
		}
		const float leafCost = C_ISECT * (float)count;
		if (count <= (uint32_t)maxLeaf && (bestAxis < 0 || leafCost <= bestCost)) { make_leaf( ni, first, count, box ); return; }
		uint32_t mid;
		if (sweepMid) mid = first + sweepMid;
		else if (bestAxis >= 0)
		{
			const float ext = cbox.hi[bestAxis] - cbox.lo[bestAxis];
			const float scale = (float)BINS * 0.99999f / ext;
			const float lo = cbox.lo[bestAxis];
			const int a = bestAxis, sb = bestBin;
			uint32_t* it = std::partition( idx.data() + first, idx.data() + first + count, [&]( uint32_t p ) {
				int b = (int)((cent[p * 3 + a] - lo) * scale);
				b = std::min( std::max( b, 0 ), BINS - 1 );
				return b <= sb;
			} );
			mid = (uint32_t)(it - idx.data());
		}
		else
		{
			/* every centroid identical (or degenerate): split the range in the middle */
			mid = first + count / 2;
		}
		if (mid == first || mid == first + count) mid = first + count / 2;
		const int c = alloc2();
		TNode& nd = nodes[ni];
		nd.box = box, nd.left = c, nd.right = c + 1, nd.first = 0, nd.count = 0;
		const uint32_t lc = mid - first, rc = count - lc;
		if (count >= PAR_THRESHOLD && threadsLeft.fetch_sub( 1 ) > 0)
		{
			std::thread t( [this, c, first, lc]() { build( c, first, lc ); } );
			build( c + 1, mid, rc );
			t.join();
			threadsLeft.fetch_add( 1 );
		}
		else
		{
			if (count >= PAR_THRESHOLD) threadsLeft.fetch_add( 1 );
			build( c, first, lc );
			build( c + 1, mid, rc );
		}
	}
};

/* ---- spatial splits (SBVH; the algorithm of Stich, Friedrich and Dietrich, "Spatial Splits in
   Bounding Volume Hierarchies", HPG 2009) -----------------------------------------------------
   A node whose best object split leaves children that overlap (overlap area > alpha x root area) also
   tries spatial splits: BINS equal slabs of the node box per axis, each reference clipped into every
   slab it crosses (the triangle polygon cut by the slab planes, intersected with the reference's
   box), entry / exit counts per slab.  A chosen spatial split sends the references that straddle the
   plane to both children, each with its clipped box, so the children do not overlap and a ray visits
   fewer of them.  A triangle then has references in several leaves: each copy is the same triangle
   record, so every leaf that a ray tests it in yields the same hit (same t, same tie rule), and the
   union of its references' boxes covers the whole triangle (the clipped boxes are widened by a few
   ulps on the axes the cut moves, and both sides of a cut include the plane). */
struct Ref { Aabb box; uint32_t prim; };

struct SpatialBuilder
{
	const float* tv = nullptr;    /* 9 floats (v0, v1, v2) per primitive */
	std::vector<TNode> nodes;
	std::vector<uint32_t> perm;   /* leaf slots, allocated per leaf (may repeat a primitive) */
	std::atomic<int> nodeCount{ 0 };
	std::atomic<uint32_t> permCount{ 0 };
	std::atomic<int64_t> refBudget{ 0 };   /* references that spatial splits may still add */
	std::atomic<int> threadsLeft{ 0 };
	int maxLeaf = 1;
	float C_TRAV = 1.0f, alpha = 1e-5f, rootArea = 1.0f;
	uint32_t minRefs = 0;         /* nodes of fewer references take the object split only */

	void make_leaf( int ni, const std::vector<Ref>& refs, const Aabb& box )
	{
		const uint32_t first = permCount.fetch_add( (uint32_t)refs.size() );
		for (size_t i = 0; i < refs.size(); i++) perm[first + i] = refs[i].prim;
		TNode& n = nodes[ni];
		n.box = box, n.left = n.right = -1, n.first = first, n.count = (uint32_t)refs.size();
	}
	static float widen( const float x ) { return std::fabs( x ) * 4e-7f + 1e-30f; }
	static bool valid( const Aabb& b ) { return b.lo[0] <= b.hi[0] && b.lo[1] <= b.hi[1] && b.lo[2] <= b.hi[2]; }
	/* the parts of reference r on either side of the plane x[a] = p */
	void split_ref( const Ref& r, const int a, const float p, Ref& L, Ref& R ) const
	{
		L.prim = R.prim = r.prim, L.box = empty_box(), R.box = empty_box();
		const float* v = tv + (size_t)r.prim * 9;
		auto add = []( Aabb& b, const float* x ) { for (int k = 0; k < 3; k++) b.lo[k] = std::min( b.lo[k], x[k] ), b.hi[k] = std::max( b.hi[k], x[k] ); };
		for (int i = 0; i < 3; i++)
		{
			const float* v0 = v + i * 3;
			const float* v1 = v + ((i + 1) % 3) * 3;
			if (v0[a] <= p) add( L.box, v0 );
			if (v0[a] >= p) add( R.box, v0 );
			if ((v0[a] < p && v1[a] > p) || (v0[a] > p && v1[a] < p))
			{
				const float t = (p - v0[a]) / (v1[a] - v0[a]);
				float x[3], lo[3], hi[3];
				for (int k = 0; k < 3; k++) x[k] = v0[k] + t * (v1[k] - v0[k]);
				for (int k = 0; k < 3; k++) lo[k] = x[k] - widen( x[k] ), hi[k] = x[k] + widen( x[k] );
				lo[a] = hi[a] = p;
				add( L.box, lo ), add( L.box, hi ), add( R.box, lo ), add( R.box, hi );
			}
		}
		/* both sides include the plane; neither leaves the reference's box */
		L.box.hi[a] = std::max( L.box.hi[a], p ), R.box.lo[a] = std::min( R.box.lo[a], p );
		for (int k = 0; k < 3; k++)
		{
			L.box.lo[k] = std::max( L.box.lo[k], r.box.lo[k] ), L.box.hi[k] = std::min( L.box.hi[k], r.box.hi[k] );
			R.box.lo[k] = std::max( R.box.lo[k], r.box.lo[k] ), R.box.hi[k] = std::min( R.box.hi[k], r.box.hi[k] );
		}
		L.box.hi[a] = std::min( L.box.hi[a], p ), R.box.lo[a] = std::max( R.box.lo[a], p );
	}

	/* the spatial binning: grows bb[b0..b1] by the box of reference r's part in each slab [lo + w b, lo + w (b + 1)]
	   of axis a (the first and last slab open towards the reference's box).  The triangle's cross-section at a
	   plane is the segment between its long edge (lowest to highest vertex on a) and the short edge on the
	   plane's side of the middle vertex; each plane's section is shared by the two slabs it bounds.  These boxes
	   only price the candidate planes (the chosen split clips with split_ref), so they are not widened. */
	void bin_slabs( const Ref& r, const int a, const float lo, const float w, const int b0, const int b1, Aabb* bb ) const
	{
		const float* v = tv + (size_t)r.prim * 9;
		const float* A = v; const float* B = v + 3; const float* C = v + 6;
		if (B[a] < A[a]) std::swap( A, B );
		if (C[a] < B[a]) std::swap( B, C );
		if (B[a] < A[a]) std::swap( A, B );
		auto lerp = []( const float* p, const float* q, const float t, float* x ) { for (int k = 0; k < 3; k++) x[k] = p[k] + t * (q[k] - p[k]); };
		auto add = []( Aabb& b, const float* x ) { for (int k = 0; k < 3; k++) b.lo[k] = std::min( b.lo[k], x[k] ), b.hi[k] = std::max( b.hi[k], x[k] ); };
		float sec[2][3];   /* the section at the slab's lower plane */
		bool haveSec = false;
		for (int b = b0; b <= b1; b++)
		{
			Aabb box = empty_box();
			const float pl = lo + w * (float)b, pu = lo + w * (float)(b + 1);
			if (haveSec) add( box, sec[0] ), add( box, sec[1] );
			for (const float* V : { A, B, C })
				if ((b == b0 || V[a] >= pl) && (b == b1 || V[a] <= pu)) add( box, V );
			haveSec = false;
			if (b < b1 && C[a] > A[a] && pu > A[a] && pu < C[a])
			{
				lerp( A, C, (pu - A[a]) / (C[a] - A[a]), sec[0] );
				if (pu < B[a]) lerp( A, B, (pu - A[a]) / (B[a] - A[a]), sec[1] );
				else if (C[a] > B[a]) lerp( B, C, (pu - B[a]) / (C[a] - B[a]), sec[1] );
				else for (int k = 0; k < 3; k++) sec[1][k] = B[k];
				sec[0][a] = sec[1][a] = pu;
				add( box, sec[0] ), add( box, sec[1] );
				haveSec = true;
			}
			for (int k = 0; k < 3; k++) box.lo[k] = std::max( box.lo[k], r.box.lo[k] ), box.hi[k] = std::min( box.hi[k], r.box.hi[k] );
			if (b > b0) box.lo[a] = std::max( box.lo[a], pl );
			if (b < b1) box.hi[a] = std::min( box.hi[a], pu );
			if (valid( box )) grow( bb[b], box );
		}
	}

	void build( int ni, std::vector<Ref>& refs )
	{
		const uint32_t count = (uint32_t)refs.size();
		Aabb box = empty_box(), cbox = empty_box();
		for (const Ref& r : refs)
		{
			grow( box, r.box );
			for (int k = 0; k < 3; k++)
			{
				const float c = 0.5f * r.box.lo[k] + 0.5f * r.box.hi[k];
				cbox.lo[k] = std::min( cbox.lo[k], c ), cbox.hi[k] = std::max( cbox.hi[k], c );
			}
		}
		if (count <= (uint32_t)std::min( 2, maxLeaf )) { make_leaf( ni, refs, box ); return; }
		const float parentArea = std::max( area( box ), 1e-30f );
		/* object split: binned SAH over the reference centroids */
		float bestCost = std::numeric_limits<float>::max();
		int bestAxis = -1, bestBin = -1;
		Aabb bestL = empty_box(), bestR = empty_box();
		for (int a = 0; a < 3; a++)
		{
			const float ext = cbox.hi[a] - cbox.lo[a];
			if (!(ext > 0)) continue;
			const float scale = (float)BINS * 0.99999f / ext;
			Aabb bb[BINS]; uint32_t bc[BINS];
			for (int b = 0; b < BINS; b++) bb[b] = empty_box(), bc[b] = 0;
			for (const Ref& r : refs)
			{
				int b = (int)(((0.5f * r.box.lo[a] + 0.5f * r.box.hi[a]) - cbox.lo[a]) * scale);
				b = std::min( std::max( b, 0 ), BINS - 1 );
				bc[b]++, grow( bb[b], r.box );
			}
			Aabb rightBox[BINS]; uint32_t rightCount[BINS];
			Aabb acc = empty_box(); uint32_t n = 0;
			for (int b = BINS - 1; b > 0; b--) { grow( acc, bb[b] ); n += bc[b]; rightBox[b] = acc, rightCount[b] = n; }
			acc = empty_box(); n = 0;
			for (int b = 0; b < BINS - 1; b++)
			{
				grow( acc, bb[b] ); n += bc[b];
				if (n == 0 || rightCount[b + 1] == 0) continue;
				const float cost = C_TRAV + C_ISECT * (area( acc ) * n + area( rightBox[b + 1] ) * rightCount[b + 1]) / parentArea;
				if (cost < bestCost) bestCost = cost, bestAxis = a, bestBin = b, bestL = acc, bestR = rightBox[b + 1];
			}
		}
		/* spatial split, where the object split's children overlap */
		int spAxis = -1;
		float spPos = 0, spCost = std::numeric_limits<float>::max();
		if (bestAxis >= 0 && count >= minRefs && refBudget.load( std::memory_order_relaxed ) > 0)
		{
			Aabb ov;
			for (int k = 0; k < 3; k++) ov.lo[k] = std::max( bestL.lo[k], bestR.lo[k] ), ov.hi[k] = std::min( bestL.hi[k], bestR.hi[k] );
			if (valid( ov ) && area( ov ) > alpha * rootArea)
			{
				for (int a = 0; a < 3; a++)
				{
					if (LH2_SBVH_AXES == 1 && a != bestAxis) continue;
					const float lo = box.lo[a], ext = box.hi[a] - lo;
					if (!(ext > 0)) continue;
					const float w = ext / (float)SBINS;
					Aabb bb[SBINS]; uint32_t entry[SBINS], exitc[SBINS];
					for (int b = 0; b < SBINS; b++) bb[b] = empty_box(), entry[b] = exitc[b] = 0;
					auto bin_of = [&]( float x ) { int b = (int)((x - lo) / w); return std::min( std::max( b, 0 ), SBINS - 1 ); };
					for (const Ref& r : refs)
					{
						const int b0 = bin_of( r.box.lo[a] ), b1 = std::max( b0, bin_of( r.box.hi[a] ) );
						entry[b0]++, exitc[b1]++;
						if (b0 == b1) grow( bb[b0], r.box );
						else bin_slabs( r, a, lo, w, b0, b1, bb );
					}
					Aabb rightBox[SBINS]; uint32_t rightCount[SBINS];
					Aabb acc = empty_box(); uint32_t n = 0;
					for (int b = SBINS - 1; b > 0; b--) { grow( acc, bb[b] ); n += exitc[b]; rightBox[b] = acc, rightCount[b] = n; }
					acc = empty_box(); n = 0;
					for (int b = 0; b < SBINS - 1; b++)
					{
						grow( acc, bb[b] ); n += entry[b];
						if (n == 0 || rightCount[b + 1] == 0) continue;
						const float cost = C_TRAV + C_ISECT * (area( acc ) * n + area( rightBox[b + 1] ) * rightCount[b + 1]) / parentArea;
						if (cost < spCost) spCost = cost, spAxis = a, spPos = lo + w * (float)(b + 1);
					}
				}
			}
		}
		const float splitCost = std::min( bestCost, spCost );
		const float leafCost = C_ISECT * (float)count;
		if (count <= (uint32_t)maxLeaf && (splitCost == std::numeric_limits<float>::max() || leafCost <= splitCost)) { make_leaf( ni, refs, box ); return; }
		std::vector<Ref> left, right;
		left.reserve( count ), right.reserve( count );
		bool spatial = spAxis >= 0 && spCost < bestCost;
		int64_t straddle = 0;
		if (spatial)
		{
			/* the straddling references come out of the duplication budget (reserved before the split) */
			for (const Ref& r : refs) straddle += r.box.lo[spAxis] < spPos && r.box.hi[spAxis] > spPos;
			if (refBudget.fetch_sub( straddle ) < straddle) refBudget.fetch_add( straddle ), spatial = false;
		}
		if (spatial)
		{
			for (const Ref& r : refs)
			{
				if (r.box.hi[spAxis] <= spPos) left.push_back( r );
				else if (r.box.lo[spAxis] >= spPos) right.push_back( r );
				else
				{
					Ref L, R;
					split_ref( r, spAxis, spPos, L, R );
					const bool lv = valid( L.box ), rv = valid( R.box );
					if (lv) left.push_back( L );
					if (rv) right.push_back( R );
					if (!lv && !rv) left.push_back( r );
				}
			}
			/* a split that does not shrink both sides could recurse forever: take the object split */
			if (left.size() >= count || right.size() >= count) left.clear(), right.clear(), spatial = false;
			/* give back the reservation the split did not use: all of it when abandoned, else the straddlers
			   whose one side clipped away */
			const int64_t added = spatial ? (int64_t)(left.size() + right.size()) - (int64_t)count : 0;
			if (straddle > added) refBudget.fetch_add( straddle - added );
		}
		if (!spatial && bestAxis >= 0)
		{
			const float ext = cbox.hi[bestAxis] - cbox.lo[bestAxis];
			const float scale = (float)BINS * 0.99999f / ext;
			for (const Ref& r : refs)
			{
				int b = (int)(((0.5f * r.box.lo[bestAxis] + 0.5f * r.box.hi[bestAxis]) - cbox.lo[bestAxis]) * scale);
				b = std::min( std::max( b, 0 ), BINS - 1 );
				(b <= bestBin ? left : right).push_back( r );
			}
		}
		if (left.empty() || right.empty())
		{
			/* every centroid identical (or degenerate): split the list in the middle */
			left.assign( refs.begin(), refs.begin() + count / 2 );
			right.assign( refs.begin() + count / 2, refs.end() );
		}
		const int c = nodeCount.fetch_add( 2 );
		TNode& nd = nodes[ni];
		nd.box = box, nd.left = c, nd.right = c + 1, nd.first = 0, nd.count = 0;
		std::vector<Ref>().swap( refs );
		if (count >= PAR_THRESHOLD && threadsLeft.fetch_sub( 1 ) > 0)
		{
			std::thread t( [this, c, &left]() { build( c, left ); } );
			build( c + 1, right );
			t.join();
			threadsLeft.fetch_add( 1 );
		}
		else
		{
			if (count >= PAR_THRESHOLD) threadsLeft.fetch_add( 1 );
			build( c, left );
			build( c + 1, right );
		}
	}
};

inline int make_leaf_ref( uint32_t first, uint32_t count ) { return (int)~((first << 4) | (count - 1)); }

/* interior nodes in DFS pre-order into the child-pair layout (lh2_device.h); leaves reference their
   ranges of out.perm */
static void Flatten( const std::vector<TNode>& tn, const float C_TRAV, BvhOutput& out )
{
	const float nanv = std::numeric_limits<float>::quiet_NaN();
	/* the leaves' primitives in DFS order (left before right), so that every subtree's leaves occupy
	   one contiguous range of out.perm (the BVH4 collapse may merge a small subtree into one leaf) */
	std::vector<uint32_t> dfsPerm;
	dfsPerm.reserve( out.perm.size() );
	std::vector<uint32_t> leafFirst( tn.size(), 0 );
	{
		std::vector<int> st{ 0 };
		while (!st.empty())
		{
			const int k = st.back();
			st.pop_back();
			const TNode& t = tn[k];
			if (t.left < 0)
			{
				leafFirst[k] = (uint32_t)dfsPerm.size();
				for (uint32_t i = 0; i < t.count; i++) dfsPerm.push_back( out.perm[t.first + i] );
				continue;
			}
			st.push_back( t.right ), st.push_back( t.left );
		}
	}
	out.perm.swap( dfsPerm );
	auto make_leaf_ref = [&]( uint32_t, uint32_t count, int k ) { return (int)~((leafFirst[k] << 4) | (count - 1)); };
	struct Item { int tnode; int gpu; int depth; };
	std::vector<Item> stack;
	auto emit = [&]() { out.nodes.resize( out.nodes.size() + 16 ); return (int)(out.nodes.size() / 16) - 1; };
	const TNode& root = tn[0];
	const float rootArea = std::max( area( root.box ), 1e-30f );
	if (root.left < 0)
	{
		const int g = emit();
		float* n = &out.nodes[(size_t)g * 16];
		n[0] = root.box.lo[0], n[1] = root.box.hi[0], n[2] = root.box.lo[1], n[3] = root.box.hi[1];
		n[4] = nanv, n[5] = nanv, n[6] = nanv, n[7] = nanv;
		n[8] = root.box.lo[2], n[9] = root.box.hi[2], n[10] = nanv, n[11] = nanv;
		int refs[4] = { make_leaf_ref( root.first, root.count, 0 ), (int)~0u, 0, 0 };
		memcpy( n + 12, refs, 16 );
		out.maxDepth = 1, out.leafCount = 1, out.sah = C_TRAV + C_ISECT * root.count;
		return;
	}
	stack.push_back( { 0, emit(), 1 } );
	double sah = 0;
	while (!stack.empty())
	{
		const Item it = stack.back();
		stack.pop_back();
		const TNode& t = tn[it.tnode];
		sah += C_TRAV * area( t.box ) / rootArea;
		out.maxDepth = std::max( out.maxDepth, it.depth );
		const TNode* ch[2] = { &tn[t.left], &tn[t.right] };
		int refs[2];
		for (int c = 0; c < 2; c++)
		{
			if (ch[c]->left < 0)
			{
				refs[c] = make_leaf_ref( ch[c]->first, ch[c]->count, c ? t.right : t.left );
				out.leafCount++;
				sah += C_ISECT * ch[c]->count * area( ch[c]->box ) / rootArea;
			}
			else refs[c] = -1;  /* patched below */
		}
		/* children pushed right-then-left so the left subtree gets the next index */
		int gidx[2] = { -1, -1 };
		for (int c = 1; c >= 0; c--) if (ch[c]->left >= 0) { gidx[c] = 0; }
		float* n;
		{
			float tmp[16];
			tmp[0] = ch[0]->box.lo[0], tmp[1] = ch[0]->box.hi[0], tmp[2] = ch[0]->box.lo[1], tmp[3] = ch[0]->box.hi[1];
			tmp[4] = ch[1]->box.lo[0], tmp[5] = ch[1]->box.hi[0], tmp[6] = ch[1]->box.lo[1], tmp[7] = ch[1]->box.hi[1];
			tmp[8] = ch[0]->box.lo[2], tmp[9] = ch[0]->box.hi[2], tmp[10] = ch[1]->box.lo[2], tmp[11] = ch[1]->box.hi[2];
			memset( tmp + 12, 0, 16 );
			n = &out.nodes[(size_t)it.gpu * 16];
			memcpy( n, tmp, 48 );
		}
		/* allocate GPU nodes for interior children: left first (DFS pre-order) */
		if (ch[0]->left >= 0) gidx[0] = emit();
		if (ch[1]->left >= 0) gidx[1] = emit();
		n = &out.nodes[(size_t)it.gpu * 16];  /* emit() may reallocate */
		for (int c = 0; c < 2; c++) if (gidx[c] >= 0) refs[c] = gidx[c];
		int r4[4] = { refs[0], refs[1], 0, 0 };
		memcpy( n + 12, r4, 16 );
		if (ch[1]->left >= 0) stack.push_back( { t.right, gidx[1], it.depth + 1 } );
		if (ch[0]->left >= 0) stack.push_back( { t.left, gidx[0], it.depth + 1 } );
	}
	out.sah = sah;
}

static void BuildSbvh( const std::vector<Aabb>& prims, int maxLeaf, int threads, BvhOutput& out, float traversalCost,
	const float* triVerts, float alpha, float budget, int minRefs )
{
	const uint32_t N = (uint32_t)prims.size();
	SpatialBuilder b;
	b.tv = triVerts, b.maxLeaf = maxLeaf, b.C_TRAV = traversalCost > 0 ? traversalCost : 1.0f, b.alpha = alpha;
	b.minRefs = (uint32_t)std::max( 0, minRefs );
	const int64_t extra = (int64_t)((double)N * std::min( budget, 4.0f ));
	b.refBudget = extra;
	const size_t maxRefs = (size_t)N + (size_t)extra;   /* splits reserve their added references first */
	b.perm.resize( maxRefs );
	b.nodes.resize( 2 * maxRefs + 1 );
	b.nodeCount = 1;
	unsigned hw = std::thread::hardware_concurrency();
	b.threadsLeft = (threads > 0 ? threads : (int)(hw ? hw : 4)) - 1;
	std::vector<Ref> refs( N );
	Aabb root = empty_box();
	for (uint32_t i = 0; i < N; i++) refs[i].box = prims[i], refs[i].prim = i, grow( root, prims[i] );
	b.rootArea = std::max( area( root ), 1e-30f );
	b.build( 0, refs );
	b.perm.resize( b.permCount.load() );
	out.nodes.clear(); out.perm = std::move( b.perm ); out.maxDepth = 0; out.leafCount = 0; out.sah = 0;
	b.nodes.resize( (size_t)b.nodeCount.load() );
	Flatten( b.nodes, b.C_TRAV, out );
}

}  // namespace

void BuildBvh2( const std::vector<Aabb>& prims, int maxLeaf, int threads, BvhOutput& out, float traversalCost, int sweepMax,
	const float* triVerts, float spatialAlpha, float spatialBudget, int spatialMinRefs )
{
	const uint32_t N = (uint32_t)prims.size();
	if (maxLeaf < 1) maxLeaf = 1;
	if (maxLeaf > 16) maxLeaf = 16;
	if (triVerts && spatialAlpha > 0 && spatialBudget > 0 && N >= 2)
	{
		BuildSbvh( prims, maxLeaf, threads, out, traversalCost, triVerts, spatialAlpha, spatialBudget, spatialMinRefs );
		return;
	}
	Builder b( prims );
	b.maxLeaf = maxLeaf;
	b.C_TRAV = traversalCost > 0 ? traversalCost : 1.0f;
	b.sweepMax = (uint32_t)std::max( 0, sweepMax );
	const float C_TRAV = b.C_TRAV;
	b.cent.resize( (size_t)N * 3 );
	b.idx.resize( N );
	for (uint32_t i = 0; i < N; i++)
	{
		b.idx[i] = i;
		for (int k = 0; k < 3; k++) b.cent[i * 3 + k] = 0.5f * prims[i].lo[k] + 0.5f * prims[i].hi[k];
	}
	b.nodes.resize( std::max<size_t>( 2 * (size_t)N + 1, 3 ) );
	b.nodeCount = 1;
	unsigned hw = std::thread::hardware_concurrency();
	b.threadsLeft = (threads > 0 ? threads : (int)(hw ? hw : 4)) - 1;
	out.nodes.clear(); out.perm.clear(); out.maxDepth = 0; out.leafCount = 0; out.sah = 0;
	const float nanv = std::numeric_limits<float>::quiet_NaN();
	if (N == 0)
	{
		/* root with two empty (NaN) children: never hit */
		out.nodes.assign( 16, nanv );
		int refs[4] = { make_leaf_ref( 0, 1 ), make_leaf_ref( 0, 1 ), 0, 0 };
		memcpy( &out.nodes[12], refs, 16 );
		return;
	}
	b.build( 0, 0, N );
	out.perm = b.idx;
	Flatten( b.nodes, C_TRAV, out );
}

/* ---- BVH2 -> BVH4 (greedy surface-area collapse) ------------------------------------------
   A BVH4 node takes a BVH2 node's two children and, while it has fewer than four, replaces its
   interior child of largest surface area by that child's two children; interior children left
   become BVH4 nodes of their own (breadth-first).  Empty (NaN-box) children are dropped; unused
   slots get NaN boxes, which no box test hits.  Leaves keep their references, so the triangle
   array (and every hit) is that of the BVH2. */
int CollapseBvh4( const float* nodes2, size_t nodeCount2, std::vector<float>& nodes4 )
{
	struct E { float lo[3], hi[3]; int ref; };
	auto children = [&]( int k, E* out ) {
		const float* n = nodes2 + (size_t)k * 16;
		int refs[2];
		memcpy( refs, n + 12, 8 );
		int m = 0;
		for (int c = 0; c < 2; c++)
		{
			E e;
			e.lo[0] = n[c * 4 + 0], e.hi[0] = n[c * 4 + 1], e.lo[1] = n[c * 4 + 2], e.hi[1] = n[c * 4 + 3];
			e.lo[2] = n[8 + c * 2], e.hi[2] = n[9 + c * 2], e.ref = refs[c];
			if (e.lo[0] == e.lo[0]) out[m++] = e;   /* NaN box: empty child */
		}
		return m;
	};
	auto area4 = [&]( const E& e ) {
		const float dx = std::max( 0.0f, e.hi[0] - e.lo[0] ), dy = std::max( 0.0f, e.hi[1] - e.lo[1] ), dz = std::max( 0.0f, e.hi[2] - e.lo[2] );
		return dx * dy + dy * dz + dz * dx;
	};
	const float nanv = std::numeric_limits<float>::quiet_NaN();
	nodes4.assign( 32, 0.0f );
	if (nodeCount2 == 0) { for (int i = 0; i < 24; i++) nodes4[i] = nanv; return 1; }
	struct Item { int node2, node4, depth; };
	std::vector<Item> queue;
	queue.push_back( { 0, 0, 1 } );
	int depth = 1;
	for (size_t qi = 0; qi < queue.size(); qi++)
	{
		const Item it = queue[qi];
		depth = std::max( depth, it.depth );
		E list[4];
		int n = children( it.node2, list );
		while (n < 4)
		{
			int best = -1;
			float bestA = -1;
			for (int i = 0; i < n; i++) if (list[i].ref >= 0 && area4( list[i] ) > bestA) best = i, bestA = area4( list[i] );
			if (best < 0) break;
			E c[2];
			const int m = children( list[best].ref, c );
			if (m == 0) { list[best] = list[--n]; continue; }
			list[best] = c[0];
			if (m == 2) list[n++] = c[1];
		}
		int refs[4] = { 0, 0, 0, 0 };
		for (int i = 0; i < n; i++)
		{
			if (list[i].ref >= 0)
			{
				const int child4 = (int)(nodes4.size() / 32);
				nodes4.resize( nodes4.size() + 32, 0.0f );
				queue.push_back( { list[i].ref, child4, it.depth + 1 } );
				refs[i] = child4;
			}
			else refs[i] = list[i].ref;
		}
		float* q = &nodes4[(size_t)it.node4 * 32];
		for (int i = 0; i < 4; i++)
		{
			/* the six planes of four (lh2_device.h): lo.x, hi.x, lo.y, hi.y, lo.z, hi.z of children 0..3 */
			const bool used = i < n;
			for (int k = 0; k < 3; k++)
				q[(2 * k) * 4 + i] = used ? list[i].lo[k] : nanv, q[(2 * k + 1) * 4 + i] = used ? list[i].hi[k] : nanv;
		}
		memcpy( q + 24, refs, 16 );
	}
	return depth;
}


/* ---- BVH2 -> W-wide by dynamic programming over the BVH2 (surface-area cost) ---------------------
   The collapse of Ylitie, Karras and Laine ("Efficient Incoherent Ray Traversal on GPUs Through
   Compressed Wide BVHs", HPG 2017, section 4) for W-wide nodes (4: the BVH4; round 5 also built an 8-wide tree with it): for every
   BVH2 subtree and every slot count j <= W, the cheapest way to hand it to a wide parent as at most j entries -
   one wide node, one leaf (a subtree of at most maxLeafTris triangles, its leaves contiguous in the DFS perm
   order that Flatten emits), or its two children's entries side by side - under the expected cost
   area x (cNode per node step, cLeaf + cTri x triangles per leaf visit).  Costs are in units of a
   node step of the traversal loop.  Output: the wide nodes in breadth-first order (node 0 the root), each a list of
   its children (ref >= 0: a wide node's index, < 0: a leaf reference as the BVH2's). */
namespace {
struct WEnt { float lo[3], hi[3]; int ref; };
int CollapseWideSah( const float* nodes2, size_t nodeCount2, const int W, float cLeaf, float cTri, int maxLeafTris,
	std::vector<std::vector<WEnt>>& wide )
{
	wide.clear();
	if (nodeCount2 == 0) { wide.emplace_back(); return 1; }
	maxLeafTris = std::min( 16, std::max( 1, maxLeafTris ) );
	const int J = W + 1;
	const float INF = std::numeric_limits<float>::infinity();
	typedef WEnt Ent;                                           /* a BVH2 child: box + reference */
	auto child = [&]( size_t k, int c, Ent& e ) {
		const float* n = nodes2 + k * 16;
		e.lo[0] = n[c * 4 + 0], e.hi[0] = n[c * 4 + 1], e.lo[1] = n[c * 4 + 2], e.hi[1] = n[c * 4 + 3];
		e.lo[2] = n[8 + c * 2], e.hi[2] = n[9 + c * 2];
		int r[2];
		memcpy( r, n + 12, 8 );
		e.ref = r[c];
		return e.lo[0] == e.lo[0];   /* NaN box: no child */
	};
	auto harea = []( const Ent& e ) {
		const float dx = std::max( 0.0f, e.hi[0] - e.lo[0] ), dy = std::max( 0.0f, e.hi[1] - e.lo[1] ), dz = std::max( 0.0f, e.hi[2] - e.lo[2] );
		return dx * dy + dy * dz + dz * dx;
	};
	/* per BVH2 node: its children, triangle count, first perm slot, and d[j] (j = 1..W) with choices */
	const size_t N2 = nodeCount2;
	std::vector<Ent> ch( N2 * 2 );
	std::vector<uint8_t> nch( N2 );
	std::vector<uint32_t> tris( N2 ), first( N2 );
	std::vector<float> d( N2 * J, INF ), asNode( N2, INF );
	std::vector<int8_t> choice( N2 * J, 0 );     /* d[j]: 0 = one entry (node or leaf), -1 = as d[j-1], i > 0: i entries to child 0 */
	std::vector<int8_t> nodeSplit( N2, 0 );      /* asNode: entries to child 0 (0: single child takes all) */
	std::vector<uint8_t> nodeCnt( N2, 0 );
	auto ent_tris = [&]( const Ent& e ) { return e.ref < 0 ? (uint32_t)(((uint32_t)(~e.ref) & 15u) + 1) : tris[e.ref]; };
	auto ent_first = [&]( const Ent& e ) { return e.ref < 0 ? (uint32_t)(~e.ref) >> 4 : first[e.ref]; };
	auto dist = [&]( const Ent& e, int j ) {
		if (e.ref < 0) return harea( e ) * (cLeaf + cTri * (float)ent_tris( e ));
		return d[(size_t)e.ref * J + j];
	};
	for (size_t kk = N2; kk-- > 0;)
	{
		int m = 0;
		for (int c = 0; c < 2; c++) { Ent e; if (child( kk, c, e )) ch[kk * 2 + m++] = e; }
		nch[kk] = (uint8_t)m;
		uint32_t t = 0, f = std::numeric_limits<uint32_t>::max();
		for (int c = 0; c < m; c++) t += ent_tris( ch[kk * 2 + c] ), f = std::min( f, ent_first( ch[kk * 2 + c] ) );
		tris[kk] = t, first[kk] = m ? f : 0;
	}
	/* the root's box: the union of its children */
	Ent rootE;
	for (int k = 0; k < 3; k++) rootE.lo[k] = INF, rootE.hi[k] = -INF;
	for (int c = 0; c < nch[0]; c++) for (int k = 0; k < 3; k++) rootE.lo[k] = std::min( rootE.lo[k], ch[c].lo[k] ), rootE.hi[k] = std::max( rootE.hi[k], ch[c].hi[k] );
	rootE.ref = 0;
	std::vector<float> area2( N2, 0.0f );
	area2[0] = harea( rootE );
	for (size_t kk = 0; kk < N2; kk++) for (int c = 0; c < nch[kk]; c++) if (ch[kk * 2 + c].ref >= 0) area2[ch[kk * 2 + c].ref] = harea( ch[kk * 2 + c] );
	/* split(k, m): the cheapest m entries made of k's children */
	auto split = [&]( size_t k, int m, int& at ) {
		float best = INF;
		at = 0;
		if (nch[k] == 1) { best = dist( ch[k * 2], m ); at = 0; return best; }
		if (nch[k] == 0) return 0.0f;
		for (int i = 1; i < m; i++)
		{
			const float c = dist( ch[k * 2], i ) + dist( ch[k * 2 + 1], m - i );
			if (c < best) best = c, at = i;
		}
		return best;
	};
	for (size_t kk = N2; kk-- > 0;)
	{
		const float A = area2[kk];
		/* as a wide node: the best 2..W entries of its children */
		float bestN = INF;
		for (int m = 2; m <= W; m++)
		{
			int at;
			const float c = split( kk, m, at );
			if (c < bestN) bestN = c, nodeSplit[kk] = (int8_t)at, nodeCnt[kk] = (uint8_t)m;
		}
		if (nch[kk] < 2) { int at; bestN = split( kk, W, at ); nodeSplit[kk] = 0, nodeCnt[kk] = (uint8_t)W; }
		asNode[kk] = A * 1.0f + bestN;
		const float asLeaf = tris[kk] <= (uint32_t)maxLeafTris && tris[kk] > 0 ? A * (cLeaf + cTri * (float)tris[kk]) : INF;
		d[kk * J + 1] = std::min( asNode[kk], asLeaf ), choice[kk * J + 1] = 0;
		for (int j = 2; j <= W; j++)
		{
			int at;
			const float c = split( kk, j, at );
			if (c < d[kk * J + j - 1]) d[kk * J + j] = c, choice[kk * J + j] = (int8_t)(nch[kk] == 1 ? 100 : at);
			else d[kk * J + j] = d[kk * J + j - 1], choice[kk * J + j] = -1;
		}
	}
	auto is_leaf_choice = [&]( size_t k ) {
		const float asLeaf = tris[k] <= (uint32_t)maxLeafTris && tris[k] > 0 ? area2[k] * (cLeaf + cTri * (float)tris[k]) : INF;
		return asLeaf < asNode[k];
	};
	/* expand(e, j): the entries that d chose for e with j slots */
	std::function<void( const Ent&, int, std::vector<Ent>& )> expand = [&]( const Ent& e, int j, std::vector<Ent>& out ) {
		if (e.ref < 0) { out.push_back( e ); return; }
		const size_t k = (size_t)e.ref;
		while (j > 1 && choice[k * J + j] == -1) j--;
		if (j == 1 || choice[k * J + j] == 0)
		{
			Ent x = e;
			if (is_leaf_choice( k )) x.ref = (int)~((first[k] << 4) | (tris[k] - 1));
			out.push_back( x );
			return;
		}
		if (choice[k * J + j] == 100) { expand( ch[k * 2], j, out ); return; }
		const int i = choice[k * J + j];
		expand( ch[k * 2], i, out );
		expand( ch[k * 2 + 1], j - i, out );
	};
	struct Item { size_t node2; int depth; };
	std::vector<Item> queue{ { 0, 1 } };
	wide.emplace_back();
	int depth = 1;
	for (size_t qi = 0; qi < queue.size(); qi++)
	{
		const Item it = queue[qi];
		depth = std::max( depth, it.depth );
		std::vector<Ent> list;
		const size_t k = it.node2;
		if (nch[k] == 1) expand( ch[k * 2], nodeCnt[k], list );
		else if (nch[k] == 2)
		{
			const int i = nodeSplit[k];
			expand( ch[k * 2], i, list );
			expand( ch[k * 2 + 1], nodeCnt[k] - i, list );
		}
		for (auto& e : list)
			if (e.ref >= 0)
			{
				queue.push_back( { (size_t)e.ref, it.depth + 1 } );
				e.ref = (int)wide.size();
				wide.emplace_back();
			}
		wide[qi] = std::move( list );
	}
	return depth;
}
}  // namespace

int CollapseBvh4Sah( const float* nodes2, size_t nodeCount2, std::vector<float>& nodes4, float cLeaf, float cTri, int maxLeafTris )
{
	const float nanv = std::numeric_limits<float>::quiet_NaN();
	nodes4.assign( 32, 0.0f );
	if (nodeCount2 == 0) { for (int i = 0; i < 24; i++) nodes4[i] = nanv; return 1; }
	std::vector<std::vector<WEnt>> wide;
	const int depth = CollapseWideSah( nodes2, nodeCount2, 4, cLeaf, cTri, maxLeafTris, wide );
	nodes4.assign( wide.size() * 32, 0.0f );
	for (size_t w = 0; w < wide.size(); w++)
	{
		const auto& list = wide[w];
		const int n = (int)list.size();
		int refs[4] = { 0, 0, 0, 0 };
		for (int i = 0; i < n; i++) refs[i] = list[i].ref;
		float* q = &nodes4[w * 32];
		for (int i = 0; i < 4; i++)
		{
			/* the six planes of four (lh2_device.h): lo.x, hi.x, lo.y, hi.y, lo.z, hi.z of children 0..3 */
			const bool used = i < n;
			for (int k = 0; k < 3; k++)
				q[(2 * k) * 4 + i] = used ? list[i].lo[k] : nanv, q[(2 * k + 1) * 4 + i] = used ? list[i].hi[k] : nanv;
		}
		memcpy( q + 24, refs, 16 );
	}
	return depth;
}

}  // namespace lh2
