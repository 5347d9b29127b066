/* lh2_bary.h - RandomBarycentrics (lights_shared.h:145-164) in closed form, shared by the shade kernels and the host checker
   (tools/bary_check.cpp).

   The reference walks 16 levels of a triangle subdivision, one base-4 digit of uf = r0 * 2^32 per level, most significant
   first: digit 1, 2, 3 keep the half-size corner triangle at A, B, C; digit 0 keeps the centre triangle, whose vertices
   are the midpoints opposite A, B, C.  It returns the final triangle's centroid as ((Ax + Bx + Cx) * 0.3333333f, ...).
   Every coordinate it computes is a dyadic rational of at most 18 significant bits, so every float operation on the way
   is exact: any exact method that yields the same vertex sums Ax + Bx + Cx and Ay + By + Cy gives bit-identical results.

   The vertex sums: with T the sum vector (start (1, 1): A = (1, 0), B = (0, 1), C = (0, 0)), o the triangle's orientation
   (+1, flipped by each digit 0) and h = o * 2^-(i+1) at level i, a digit 1 adds (2h, -h), a digit 2 (-h, 2h), a digit 3
   (-h, -h) (the centroid moves halfway toward the kept corner), a digit 0 adds nothing.  In units of 2^-17, per digit i at
   bit position p = 15 - i of the 16-bit digit masks (weight 2^p, h = +-2^(p+1)):
     Tx = 2^17 + 4 (D1 & P) - 4 (D1 & N) - 2 (H & P) + 2 (H & N)
     Ty = 2^17 - 2 (L & P) + 2 (L & N) + 4 (D2 & P) - 4 (D2 & N)
   L / H the digits' low / high bits, D1 = L & ~H, D2 = H & ~L, N the levels below an odd number of 0 digits, P the rest
   (a prefix parity, from the most significant level).  About 45 integer instructions instead of the loop's 16 four-way
   branches (~600 VALU instructions per call in the shade kernels, all four branches executed by divergent lanes). */
#pragma once
#include <stdint.h>
#if defined( __HIP__ )
#include <hip/hip_runtime.h>
#define LH2_BARY_HD __host__ __device__
#else
#define LH2_BARY_HD
#endif

/* the 16 bits at even positions of x, packed (bit 2k -> bit k) */
LH2_BARY_HD inline uint32_t lh2_even_bits( uint32_t x )
{
	x &= 0x55555555u;
	x = (x | (x >> 1)) & 0x33333333u;
	x = (x | (x >> 2)) & 0x0F0F0F0Fu;
	x = (x | (x >> 4)) & 0x00FF00FFu;
	return (x | (x >> 8)) & 0x0000FFFFu;
}

/* the vertex sums Ax + Bx + Cx, Ay + By + Cy of the reference's final triangle for the digit string uf, exactly */
LH2_BARY_HD inline void lh2_bary_sums( const uint32_t uf, float& sx, float& sy )
{
	const uint32_t L = lh2_even_bits( uf ), H = lh2_even_bits( uf >> 1 );
	const uint32_t D1 = L & ~H, D2 = H & ~L, Z = ~(L | H) & 0xFFFFu;
	/* Q bit p: parity of the 0 digits at levels above p (bits p + 1 .. 15 of Z) */
	uint32_t Q = Z >> 1;
	Q ^= Q >> 1, Q ^= Q >> 2, Q ^= Q >> 4, Q ^= Q >> 8;
	const uint32_t N = Q & 0xFFFFu, P = ~Q & 0xFFFFu;
	const int32_t tx = (1 << 17) + 4 * (int32_t)(D1 & P) - 4 * (int32_t)(D1 & N) - 2 * (int32_t)(H & P) + 2 * (int32_t)(H & N);
	const int32_t ty = (1 << 17) - 2 * (int32_t)(L & P) + 2 * (int32_t)(L & N) + 4 * (int32_t)(D2 & P) - 4 * (int32_t)(D2 & N);
	sx = (float)tx * 7.62939453125e-06f, sy = (float)ty * 7.62939453125e-06f;   /* exact: |t| < 2^24, times 2^-17 */
}
