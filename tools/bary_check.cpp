/* bary_check.cpp - host check (tests/test_bary.py): lh2_bary.h's closed-form RandomBarycentrics against the reference loop
   (lights_shared.h:145-164, restated here as the oracle restates it) for the given uf values: a strided sweep of the 2^32
   digit strings plus every string whose digits are all equal in two runs, bit for bit on the returned (rx, ry, 1 - rx - ry).
   Build: g++ -O2 -std=c++17 -ffp-contract=off tools/bary_check.cpp -o /tmp/bary_check; run: /tmp/bary_check [stride] */
#include "../lighthouse2_amd/csrc/lh2_bary.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

static void reference( const uint32_t uf, float& rx, float& ry )
{
	float Ax = 1, Ay = 0, Bx = 0, By = 1, Cx = 0, Cy = 0;
	for (int i = 0; i < 16; ++i)
	{
		const int d = (uf >> (2 * (15 - i))) & 0x3;
		float Anx, Any, Bnx, Bny, Cnx, Cny;
		switch (d)
		{
		case 0: Anx = (Bx + Cx) * 0.5f, Any = (By + Cy) * 0.5f; Bnx = (Ax + Cx) * 0.5f, Bny = (Ay + Cy) * 0.5f; Cnx = (Ax + Bx) * 0.5f, Cny = (Ay + By) * 0.5f; break;
		case 1: Anx = Ax, Any = Ay; Bnx = (Ax + Bx) * 0.5f, Bny = (Ay + By) * 0.5f; Cnx = (Ax + Cx) * 0.5f, Cny = (Ay + Cy) * 0.5f; break;
		case 2: Anx = (Bx + Ax) * 0.5f, Any = (By + Ay) * 0.5f; Bnx = Bx, Bny = By; Cnx = (Bx + Cx) * 0.5f, Cny = (By + Cy) * 0.5f; break;
		default: Anx = (Cx + Ax) * 0.5f, Any = (Cy + Ay) * 0.5f; Bnx = (Cx + Bx) * 0.5f, Bny = (Cy + By) * 0.5f; Cnx = Cx, Cny = Cy; break;
		}
		Ax = Anx, Ay = Any, Bx = Bnx, By = Bny, Cx = Cnx, Cy = Cny;
	}
	rx = (Ax + Bx + Cx) * 0.3333333f, ry = (Ay + By + Cy) * 0.3333333f;
}

static bool same( float a, float b ) { uint32_t x, y; memcpy( &x, &a, 4 ), memcpy( &y, &b, 4 ); return x == y; }

static int check( uint32_t uf, long& bad )
{
	float rx, ry, sx, sy;
	reference( uf, rx, ry );
	lh2_bary_sums( uf, sx, sy );
	const float fx = sx * 0.3333333f, fy = sy * 0.3333333f;
	if (!same( rx, fx ) || !same( ry, fy ) || !same( 1 - rx - ry, 1 - fx - fy ))
	{
		if (bad++ < 5) printf( "mismatch uf %08x: ref %.9g %.9g fast %.9g %.9g\n", uf, rx, ry, fx, fy );
		return 1;
	}
	return 0;
}

int main( int argc, char** argv )
{
	const uint64_t stride = argc > 1 ? strtoull( argv[1], nullptr, 0 ) : 257;
	long bad = 0, n = 0;
	for (uint64_t u = 0; u < (1ull << 32); u += stride) check( (uint32_t)u, bad ), n++;
	/* runs of equal digits split at every level */
	for (int a = 0; a < 4; a++) for (int b = 0; b < 4; b++) for (int k = 0; k <= 16; k++)
	{
		uint32_t uf = 0;
		for (int i = 0; i < 16; i++) uf |= (uint32_t)(i < k ? a : b) << (2 * (15 - i));
		check( uf, bad ), n++;
	}
	check( 0xFFFFFFFFu, bad ), n++;
	printf( "{\"checked\": %ld, \"mismatches\": %ld}\n", n, bad );
	return bad ? 1 : 0;
}
