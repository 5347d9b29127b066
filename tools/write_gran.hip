// Calibration of rocprofv3's WRITE_SIZE for the closest-hit launch's store pattern (the
// bounce launch reports ~34 B written per ray against its 16-B hit record).  The traversal stores one
// uint4 per finished ray at the ray's index, at the time the ray finishes: neighbouring records are
// written by different lanes / waves at different times.  Three launches write the same 2^21 records:
//   coalesced  - lane i stores record i (a wave writes 1 KiB contiguous)
//   scattered  - lane i stores record perm[i], perm a random permutation of all records
//   windowed   - perm random within windows of 4096 records (a segment's refill batches finishing out of order)
// Run under `rocprofv3 --pmc WRITE_SIZE --kernel-trace` and divide by the 32 MiB written.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/write_gran tools/write_gran.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

#define CHECK( x ) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf( stderr, "%s: %s\n", #x, hipGetErrorString( e_ ) ); exit( 1 ); } } while (0)

__global__ void k_coalesced( uint4* out, uint32_t n )
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = make_uint4( i, i * 3u, i ^ 0x5555u, 7u );
}

__global__ void k_permuted( uint4* out, const uint32_t* perm, uint32_t n )
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) { const uint32_t j = perm[i]; out[j] = make_uint4( j, j * 3u, j ^ 0x5555u, 7u ); }
}

int main()
{
	const uint32_t n = 1u << 21;
	std::vector<uint32_t> scattered( n ), windowed( n );
	for (uint32_t i = 0; i < n; i++) scattered[i] = windowed[i] = i;
	std::mt19937 rng( 1 );
	std::shuffle( scattered.begin(), scattered.end(), rng );
	for (uint32_t w = 0; w < n; w += 4096) std::shuffle( windowed.begin() + w, windowed.begin() + std::min( n, w + 4096 ), rng );
	uint4* out; uint32_t *dS, *dW;
	CHECK( hipMalloc( &out, (size_t)n * 16 ) );
	CHECK( hipMalloc( &dS, (size_t)n * 4 ) );
	CHECK( hipMalloc( &dW, (size_t)n * 4 ) );
	CHECK( hipMemcpy( dS, scattered.data(), (size_t)n * 4, hipMemcpyHostToDevice ) );
	CHECK( hipMemcpy( dW, windowed.data(), (size_t)n * 4, hipMemcpyHostToDevice ) );
	const uint32_t blocks = (n + 255) / 256;
	for (int rep = 0; rep < 3; rep++)
	{
		k_coalesced<<<blocks, 256>>>( out, n );
		k_permuted<<<blocks, 256>>>( out, dS, n );
		k_permuted<<<blocks, 256>>>( out, dW, n );
	}
	CHECK( hipDeviceSynchronize() );
	std::vector<uint4> h( n );
	CHECK( hipMemcpy( h.data(), out, (size_t)n * 16, hipMemcpyDeviceToHost ) );
	uint32_t bad = 0;
	for (uint32_t i = 0; i < n; i++) bad += h[i].x != i || h[i].w != 7u;
	printf( "{\"records\": %u, \"bytes\": %zu, \"bad\": %u, \"launches\": [\"coalesced\", \"scattered\", \"windowed4096\"]}\n", n, (size_t)n * 16, bad );
	CHECK( hipFree( out ) ); CHECK( hipFree( dS ) ); CHECK( hipFree( dW ) );
	return bad != 0;
}
