/* lh2_w8.h - the 8-wide compressed BVH ("W8", round 5): record format, slot assignment and quantizer, shared by the host
   builder (bvh_build.cpp BuildW8), the per-frame TLAS conversion (bvh_gpu.hip k_tlas_to_w8) and the traversal
   (lh2_trace4d.inc, WIDE).

   After Ylitie, Karras and Laine, "Efficient Incoherent Ray Traversal on GPUs Through Compressed Wide BVHs" (HPG 2017):
   a node's children live side by side in a block of 8 records (a child's record index = 8 x the parent's child block +
   its slot), so the traversal stack holds one entry per node step - a node group, (child block, the slots still to visit)
   - instead of one reference per child, and needs no sort: a child's slot is assigned at build time by the direction of
   its centroid from the parent's centre (slot bit k set: the child lies on the negative side of axis k), and a ray visits
   the slots in the order of slot ^ m, m its direction's octant (bit k: d_k > 0), nearest corner first.

   Records are 80 B (LH2_W8_WORDS u32), an array of blocks of 8 (SceneDev::w8):
     node      u32[0..2]   origin x, y, z (f32: the children's union low corner)
               u32[3]      grid exponents e_x, e_y, e_z (signed bytes, plane = origin + q * 2^e), byte 3 = 0
               u32[4..15]  child planes as bytes, slots 0..3 in the first word of each pair, 4..7 in the second:
                           x lo (4, 5), x hi (6, 7), y lo (8, 9), y hi (10, 11), z lo (12, 13), z hi (14, 15)
               u32[16..17] the interior children's slot mask in key order for each ray octant m (byte m: bit k set
                           when slot k ^ m holds an interior node), so a node step splits its hits into node and leaf
                           children with one byte select
               u32[18]     the child block (a BLAS: relative to its mesh's first block; the TLAS: absolute)
               u32[19]     0
     triangle  u32[0..11]  a BLAS leaf (one triangle): the 48-B triangle record of lh2_device.h
     instance  u32[0..11]  a TLAS leaf: the instance's inverse rows 0..2 (DevInstance), u32[12] its index, u32[13] its
                           mesh's first block
   An empty slot has the inverted box (lo 255, hi 0), which no ray enters.  Planes round outward exactly as the BVH4
   quantizer's (bvh_gpu.hip k_quantize4): the quantized box holds the f32 one, so the box tests only cull and every hit
   is the BVH2's. */
#pragma once
#if defined( __HIP__ )
#include <hip/hip_runtime.h>
#define LH2_W8_HD __host__ __device__
#else
#define LH2_W8_HD   /* a plain C++ compiler (the host checkers, tools/w8_check.cpp) */
#endif
#include <stdint.h>
#include <math.h>

#define LH2_W8_WORDS 20
#define LH2_W8_BYTES 80
/* the largest grid exponent (box4q / box8q scale the ray's clamped reciprocal +-1e30 by 2^e: 1e30 * 2^27 stays finite) */
#define LH2_QEXP_MAX 27
/* a traversal stack entry of the wide loop: child block << 9 | leaf group (0x100) | the slots still to visit in key order;
   the block stays below 2^22 - 1 so that ~entry (a leaf group waiting in `node`) is negative and never the pop / finish
   markers */
#define LH2_W8_MAX_BLOCKS ((1u << 22) - 2u)

/* the slots of n <= 8 children by the directions of their centroids from the parent's centre (d[i]): greedily the
   (child, slot) pairs of the largest d . diag(slot), diag(slot)_k = -1 when bit k of slot is set, else +1 */
LH2_W8_HD inline void lh2_w8_assign( const int n, const float d[8][3], int slotOf[8] )
{
	bool used[8] = {}, done[8] = {};
	for (int i = 0; i < 8; i++) slotOf[i] = -1;
	for (int r = 0; r < n; r++)
	{
		float best = -INFINITY;
		int bi = -1, bs = -1;
		for (int i = 0; i < n; i++)
		{
			if (done[i]) continue;
			for (int s = 0; s < 8; s++)
			{
				if (used[s]) continue;
				const float v = ((s & 1) ? -d[i][0] : d[i][0]) + ((s & 2) ? -d[i][1] : d[i][1]) + ((s & 4) ? -d[i][2] : d[i][2]);
				if (bi < 0 || v > best) best = v, bi = i, bs = s;
			}
		}
		done[bi] = true, used[bs] = true, slotOf[bi] = bs;
	}
}

/* the interior-slot masks in key order (u32[16..17]): byte m, bit k = slot k ^ m is interior */
LH2_W8_HD inline void lh2_w8_imask_keys( const uint32_t imask, uint32_t& lo, uint32_t& hi )
{
	lo = hi = 0;
	for (uint32_t m = 0; m < 8; m++)
	{
		uint32_t b = 0;
		for (uint32_t k = 0; k < 8; k++) if ((imask >> (k ^ m)) & 1u) b |= 1u << k;
		if (m < 4) lo |= b << (8 * m); else hi |= b << (8 * (m - 4));
	}
}

/* one node record's words 0..17 from the children by slot (valid[s]: slot s holds a child with the box lo / hi) and the
   interior slots; returns nonzero when a child box needs a grid exponent beyond LH2_QEXP_MAX (LH2_SCENE_ERR_QRANGE) */
LH2_W8_HD inline int lh2_w8_quantize( const bool valid[8], const float lo[8][3], const float hi[8][3], const uint32_t imask,
	uint32_t* rec )
{
	int err = 0;
	uint32_t qlo[3][2] = {}, qhi[3][2] = {};
	float origin[3];
	int e[3];
	for (int a = 0; a < 3; a++)
	{
		float o = 0, mx = 0;
		bool any = false;
		for (int c = 0; c < 8; c++)
			if (valid[c]) o = any ? fminf( o, lo[c][a] ) : lo[c][a], mx = any ? fmaxf( mx, hi[c][a] ) : hi[c][a], any = true;
		origin[a] = o;
		const double ext = (double)mx - (double)o;
		const double mag = fmax( fabs( (double)o ), fabs( (double)mx ) );
		int ea = -100;
		if (ext > 0) { const int c = (int)ceil( log2( ext / 255.0 ) ); ea = c > ea ? c : ea; }
		if (mag > 0) { const int c = (int)floor( log2( mag ) ) - 28; ea = c > ea ? c : ea; }
		while (ext > 255.0 * ldexp( 1.0, ea ) && ea <= LH2_QEXP_MAX) ea++;
		if (ea > LH2_QEXP_MAX) err = 1, ea = LH2_QEXP_MAX;
		e[a] = ea;
		const double step = ldexp( 1.0, ea );
		for (int c = 0; c < 8; c++)
		{
			uint32_t l = 255, h = 0;
			if (valid[c])
			{
				const double dl = floor( ((double)lo[c][a] - (double)o) / step ), dh = ceil( ((double)hi[c][a] - (double)o) / step );
				l = (uint32_t)fmin( fmax( dl, 0.0 ), 255.0 ), h = (uint32_t)fmin( fmax( dh, 0.0 ), 255.0 );
				while (l > 0 && (double)o + (double)l * step > (double)lo[c][a]) l--;
				while (h < 255 && (double)o + (double)h * step < (double)hi[c][a]) h++;
			}
			qlo[a][c >> 2] |= l << (8 * (c & 3)), qhi[a][c >> 2] |= h << (8 * (c & 3));
		}
	}
	union { float f; uint32_t u; } cv;
	for (int a = 0; a < 3; a++) cv.f = origin[a], rec[a] = cv.u;
	rec[3] = (uint32_t)(e[0] & 255) | ((uint32_t)(e[1] & 255) << 8) | ((uint32_t)(e[2] & 255) << 16);
	for (int a = 0; a < 3; a++) rec[4 + 4 * a] = qlo[a][0], rec[5 + 4 * a] = qlo[a][1], rec[6 + 4 * a] = qhi[a][0], rec[7 + 4 * a] = qhi[a][1];
	lh2_w8_imask_keys( imask, rec[16], rec[17] );
	return err;
}

/* a child box is one: finite, lo <= hi on every axis (NaN boxes mark absent BVH2 children) */
LH2_W8_HD inline bool lh2_w8_box_valid( const float lo[3], const float hi[3] )
{
	for (int a = 0; a < 3; a++) if (!(isfinite( lo[a] ) && isfinite( hi[a] ) && lo[a] <= hi[a])) return false;
	return true;
}
