/* lh2_detmath.h - deterministic fp32 elementary functions (the parity numerics contract).

   The reference render core (RenderCore_OptixPrime_B) was built with nvcc --use_fast_math
   (rendercore_optixprime_b.vcxproj FastMath=true), so its __sincosf / __expf / atan2 / acos
   values are device approximations that no CPU libm reproduces.  Parity between the HIP core
   and the CPU oracle therefore needs ONE definition of every transcendental the hot path uses
   (SURVEY.md §8 (c') "Parity-critical numerics").  This header is that definition: Cephes-style
   range reduction + minimax polynomials (S. Moshier, Cephes Math Library, public algorithms)
   written with only IEEE +,-,*,/ and sqrt, so that gcc (-ffp-contract=off) on the host and
   hipcc (-ffp-contract=off) for gfx950 produce bit-identical results.

   Users:  lighthouse2_amd/csrc HIP sources (product)  and  oracle/pt_oracle.c (CPU restatement).
   Accuracy vs libm is tested in tests/test_detmath.py (a few ulp; the reference's fast-math
   intrinsics are far looser).

   Compile rule: every includer MUST build with -ffp-contract=off (no FMA contraction), and
   without -ffast-math.
*/
#ifndef LH2_DETMATH_H
#define LH2_DETMATH_H

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
#define LH2_DM_FN static __host__ __device__ inline
#else
#define LH2_DM_FN static inline
#endif

#ifdef __cplusplus
#include <cmath>
#include <cstdint>
#include <cstring>
#define LH2_DM_SQRTF(x) sqrtf(x)
#define LH2_DM_FLOORF(x) floorf(x)
#else
#include <math.h>
#include <stdint.h>
#include <string.h>
#define LH2_DM_SQRTF(x) sqrtf(x)
#define LH2_DM_FLOORF(x) floorf(x)
#endif

#define LH2_PI      3.14159265358979323846264f
#define LH2_INVPI   0.31830988618379067153777f
#define LH2_TWOPI   6.28318530717958647692528f
#define LH2_PIO2    1.57079632679489661923132f
#define LH2_PIO4    0.78539816339744830961566f

LH2_DM_FN uint32_t lh2_f2b( float f ) { uint32_t u; memcpy( &u, &f, 4 ); return u; }
LH2_DM_FN float lh2_b2f( uint32_t u ) { float f; memcpy( &f, &u, 4 ); return f; }

/* float -> uint32 with the saturating semantics of the GPU convert instruction
   (v_cvt_u32_f32 / NVIDIA cvt.rzi.u32.f32): NaN -> 0, x <= 0 -> 0, x >= 2^32 -> 0xffffffff,
   otherwise truncation toward zero.  A plain C cast is UB outside [0, 2^32) and differs
   between x86 and the GPU, so every float->uint in the hot path goes through this. */
LH2_DM_FN uint32_t lh2_f2u( float x )
{
	if (!(x > 0.0f)) return 0u;               /* also catches NaN */
	if (x >= 4294967296.0f) return 0xffffffffu;
	return (uint32_t)x;
}
/* float -> int32, saturating, NaN -> 0 (v_cvt_i32_f32 semantics). */
LH2_DM_FN int32_t lh2_f2i( float x )
{
	if (x != x) return 0;
	if (x >= 2147483648.0f) return 2147483647;
	if (x <= -2147483648.0f) return (int32_t)0x80000000u;
	return (int32_t)x;
}

/* 2^n for integer n in [-126, 127] (exact, built from the exponent bits). */
LH2_DM_FN float lh2_exp2i( int n ) { return lh2_b2f( (uint32_t)(n + 127) << 23 ); }

/* ---- sine / cosine: Cody-Waite reduction by pi/2, Cephes sinf/cosf kernels ---------- */
/* pi/2 split so that k*PIO2_A and k*PIO2_B are exact for |k| < 2^11 */
#define LH2_PIO2_A 1.5703125f                 /* 12 significant bits */
#define LH2_PIO2_B 4.837512969970703125e-4f   /* next 12 bits */
#define LH2_PIO2_C 7.549789948768648e-8f      /* remainder */
LH2_DM_FN float lh2_sin_kernel( float r ) /* |r| <= pi/4 */
{
	const float z = r * r;
	return ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
}
LH2_DM_FN float lh2_cos_kernel( float r )
{
	const float z = r * r;
	float y = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z;
	y = y - 0.5f * z;
	return y + 1.0f;
}
LH2_DM_FN void lh2_sincosf( float x, float* s, float* c )
{
	if (!(x == x) || x - x != 0.0f) { *s = x - x; *c = x - x; return; } /* NaN / inf -> NaN */
	const float kf = LH2_DM_FLOORF( x * 0.63661977236758134308f + 0.5f );
	const int k = (int)kf;
	const float r = ((x - kf * LH2_PIO2_A) - kf * LH2_PIO2_B) - kf * LH2_PIO2_C;
	const float sr = lh2_sin_kernel( r ), cr = lh2_cos_kernel( r );
	switch (k & 3)
	{
	case 0: *s = sr; *c = cr; break;
	case 1: *s = cr; *c = -sr; break;
	case 2: *s = -sr; *c = -cr; break;
	default: *s = -cr; *c = sr; break;
	}
}
LH2_DM_FN float lh2_sinf( float x ) { float s, c; lh2_sincosf( x, &s, &c ); return s; }
LH2_DM_FN float lh2_cosf( float x ) { float s, c; lh2_sincosf( x, &s, &c ); return c; }

/* ---- exp: Cephes expf ----------------------------------------------------------------- */
LH2_DM_FN float lh2_expf( float x )
{
	if (x != x) return x;
	if (x > 88.72283905206835f) return lh2_b2f( 0x7f800000u );
	if (x < -87.33654475055310f) return 0.0f;
	const float nf = LH2_DM_FLOORF( x * 1.44269504088896341f + 0.5f );
	const float r = (x - nf * 0.693359375f) - nf * -2.12194440e-4f;
	const float z = r * r;
	float y = ((((( 1.9875691500e-4f * r + 1.3981999507e-3f) * r + 8.3334519073e-3f) * r
		+ 4.1665795894e-2f) * r + 1.6666665459e-1f) * r + 5.0000001201e-1f) * z + r + 1.0f;
	int n = (int)nf;
	/* y in ~[0.7, 1.42]; split the scale so both factors are normal */
	if (n > 127) { y = y * 2.0f; n -= 1; }
	if (n < -126) { y = y * lh2_exp2i( -126 ); n += 126; }
	return y * lh2_exp2i( n );
}

/* ---- log: Cephes logf ----------------------------------------------------------------- */
LH2_DM_FN float lh2_logf( float x )
{
	if (x != x) return x;
	if (x < 0.0f) return lh2_b2f( 0x7fc00000u );
	if (x == 0.0f) return lh2_b2f( 0xff800000u );
	if (x - x != 0.0f) return x; /* +inf */
	int e = 0;
	if (x < 1.17549435e-38f) { x = x * 16777216.0f; e = -24; }  /* denormal: scale by 2^24 */
	uint32_t u = lh2_f2b( x );
	e += (int)((u >> 23) & 255u) - 126;
	float m = lh2_b2f( (u & 0x007fffffu) | 0x3f000000u ); /* [0.5, 1) */
	if (m < 0.70710678118654752440f) { e -= 1; m = m + m - 1.0f; } else m = m - 1.0f;
	const float z = m * m;
	float y = ((((((((7.0376836292e-2f * m - 1.1514610310e-1f) * m + 1.1676998740e-1f) * m
		- 1.2420140846e-1f) * m + 1.4249322787e-1f) * m - 1.6668057665e-1f) * m
		+ 2.0000714765e-1f) * m - 2.4999993993e-1f) * m + 3.3333331174e-1f) * m * z;
	const float fe = (float)e;
	y = y + fe * -2.12194440e-4f;
	y = y - 0.5f * z;
	return (m + y) + fe * 0.693359375f;
}
LH2_DM_FN float lh2_log2f( float x ) { return lh2_logf( x ) * 1.44269504088896341f; }

/* ---- pow for x > 0 (the hot path only raises positive bases) --------------------------- */
LH2_DM_FN float lh2_powf( float x, float y )
{
	if (y == 0.0f) return 1.0f;
	if (x == 0.0f) return y > 0.0f ? 0.0f : lh2_b2f( 0x7f800000u );
	if (x == 1.0f) return 1.0f;
	return lh2_expf( y * lh2_logf( x ) );
}

/* ---- atan / atan2: Cephes atanf -------------------------------------------------------- */
LH2_DM_FN float lh2_atanf( float x )
{
	if (x != x) return x;
	float sgn = 1.0f;
	if (x < 0.0f) { sgn = -1.0f; x = -x; }
	float y0;
	if (x > 2.414213562373095f) { y0 = LH2_PIO2; x = -1.0f / x; }
	else if (x > 0.4142135623730950f) { y0 = LH2_PIO4; x = (x - 1.0f) / (x + 1.0f); }
	else y0 = 0.0f;
	const float z = x * x;
	const float y = (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z
		- 3.33329491539e-1f) * z * x + x;
	return sgn * (y0 + y);
}
LH2_DM_FN float lh2_atan2f( float y, float x )
{
	if (x != x || y != y) return x + y;
	if (x == 0.0f)
	{
		if (y > 0.0f) return LH2_PIO2;
		if (y < 0.0f) return -LH2_PIO2;
		return 0.0f;
	}
	if (y == 0.0f) return x > 0.0f ? 0.0f : LH2_PI;
	const float z = lh2_atanf( y / x );
	if (x > 0.0f) return z;
	return y > 0.0f ? z + LH2_PI : z - LH2_PI;
}

/* ---- asin / acos: Cephes asinf --------------------------------------------------------- */
LH2_DM_FN float lh2_asinf( float x )
{
	if (!(x >= -1.0f && x <= 1.0f)) return lh2_b2f( 0x7fc00000u );
	float sgn = 1.0f, a = x;
	if (a < 0.0f) { sgn = -1.0f; a = -a; }
	float z, r;
	int flag = 0;
	if (a > 0.5f) { z = 0.5f * (1.0f - a); r = LH2_DM_SQRTF( z ); flag = 1; }
	else { z = a * a; r = a; }
	float y = ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z
		+ 7.4953002686e-2f) * z + 1.6666752422e-1f) * z * r + r;
	if (flag) { y = y + y; y = LH2_PIO2 - y; }
	return sgn * y;
}
LH2_DM_FN float lh2_acosf( float x )
{
	if (!(x >= -1.0f && x <= 1.0f)) return lh2_b2f( 0x7fc00000u );
	if (x < -0.5f) return LH2_PI - 2.0f * lh2_asinf( LH2_DM_SQRTF( 0.5f * (1.0f + x) ) );
	if (x > 0.5f) return 2.0f * lh2_asinf( LH2_DM_SQRTF( 0.5f * (1.0f - x) ) );
	return LH2_PIO2 - lh2_asinf( x );
}

/* ---- IEEE half (binary16) round-to-nearest-even, as half.hpp does on the host ---------- */
LH2_DM_FN uint16_t lh2_f2h( float f )
{
	const uint32_t u = lh2_f2b( f );
	const uint32_t sign = (u >> 16) & 0x8000u;
	const uint32_t absu = u & 0x7fffffffu;
	if (absu >= 0x7f800000u) return (uint16_t)(sign | (absu > 0x7f800000u ? 0x7e00u : 0x7c00u));
	if (absu >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520 -> inf */
	if (absu < 0x38800000u)
	{
		/* half subnormal or zero: value = absu-float; half ulp = 2^-24 */
		if (absu < 0x33000000u) return (uint16_t)sign; /* < 2^-25 -> 0 (ties at 2^-25 -> 0) */
		const uint32_t e = absu >> 23;
		const uint32_t mant = (absu & 0x7fffffu) | 0x800000u;
		const uint32_t shift = 126u - e; /* 14..24 */
		uint32_t h = mant >> shift;
		const uint32_t rem = mant & ((1u << shift) - 1u);
		const uint32_t halfway = 1u << (shift - 1u);
		if (rem > halfway || (rem == halfway && (h & 1u))) h++;
		return (uint16_t)(sign | h);
	}
	uint32_t h = ((absu - 0x38000000u) >> 13);
	const uint32_t rem = absu & 0x1fffu;
	if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
	return (uint16_t)(sign | h);
}
LH2_DM_FN float lh2_h2f( uint16_t h )
{
	const uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
	uint32_t e = ((uint32_t)h >> 10) & 31u, m = (uint32_t)h & 1023u;
	if (e == 31u) return lh2_b2f( sign | 0x7f800000u | (m << 13) );
	if (e == 0u)
	{
		if (m == 0u) return lh2_b2f( sign );
		/* subnormal: m * 2^-24 (exact in float) */
		const float v = (float)m * 5.9604644775390625e-8f;
		return sign ? -v : v;
	}
	return lh2_b2f( sign | ((e + 112u) << 23) | (m << 13) );
}

#endif /* LH2_DETMATH_H */
