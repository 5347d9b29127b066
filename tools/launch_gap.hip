/* launch_gap.hip - the cost of a dependent launch on one stream, by launch flavour (tools only).
   N launches of a small kernel (1024 x 256 threads, one store each), each mode timed with events
   around the whole batch:
     plain    hipLaunchKernelGGL
     stop     hipExtLaunchKernelGGL with a stop event (what the core uses for its per-pass times)
     startstop  ... with start and stop events
     record   plain launch + hipEventRecord after it
     graph    the plain batch captured once into a hipGraph, then hipGraphLaunch
   Build: hipcc -O3 --offload-arch=gfx950 tools/launch_gap.hip -o tools/launch_gap */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

#define CK( x ) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf( "HIP error %s at %d\n", hipGetErrorString( e_ ), __LINE__ ); return 1; } } while (0)

__global__ void k_small( float* p, int i )
{
	const int t = blockIdx.x * blockDim.x + threadIdx.x;
	p[t] = p[t] * 0.5f + (float)i;
}

int main()
{
	const int N = 2000, G = 1024, B = 256;
	float* d = nullptr;
	CK( hipMalloc( &d, sizeof( float ) * G * B ) );
	CK( hipMemset( d, 0, sizeof( float ) * G * B ) );
	hipStream_t st;
	CK( hipStreamCreateWithFlags( &st, hipStreamNonBlocking ) );
	std::vector<hipEvent_t> ev( 2 * N );
	for (auto& e : ev) CK( hipEventCreate( &e ) );
	hipEvent_t a, b;
	CK( hipEventCreate( &a ) );
	CK( hipEventCreate( &b ) );
	const char* names[] = { "plain", "stop", "startstop", "record", "graph" };
	hipGraphExec_t exec = nullptr;
	for (int mode = 0; mode < 5; mode++)
	{
		if (mode == 4)
		{
			hipGraph_t g;
			CK( hipStreamBeginCapture( st, hipStreamCaptureModeGlobal ) );
			for (int i = 0; i < N; i++) hipLaunchKernelGGL( k_small, dim3( G ), dim3( B ), 0, st, d, i );
			CK( hipStreamEndCapture( st, &g ) );
			CK( hipGraphInstantiate( &exec, g, nullptr, nullptr, 0 ) );
			CK( hipGraphLaunch( exec, st ) );   /* warm */
		}
		for (int rep = 0; rep < 3; rep++)
		{
			CK( hipStreamSynchronize( st ) );
			CK( hipEventRecord( a, st ) );
			if (mode == 4) CK( hipGraphLaunch( exec, st ) );
			else for (int i = 0; i < N; i++)
			{
				if (mode == 0) hipLaunchKernelGGL( k_small, dim3( G ), dim3( B ), 0, st, d, i );
				else if (mode == 1) hipExtLaunchKernelGGL( k_small, dim3( G ), dim3( B ), 0, st, nullptr, ev[i], 0, d, i );
				else if (mode == 2) hipExtLaunchKernelGGL( k_small, dim3( G ), dim3( B ), 0, st, ev[N + i], ev[i], 0, d, i );
				else { hipLaunchKernelGGL( k_small, dim3( G ), dim3( B ), 0, st, d, i ); CK( hipEventRecord( ev[i], st ) ); }
			}
			CK( hipEventRecord( b, st ) );
			CK( hipEventSynchronize( b ) );
			float ms = 0;
			CK( hipEventElapsedTime( &ms, a, b ) );
			if (rep == 2) std::printf( "{\"mode\": \"%s\", \"launches\": %d, \"us_per_launch\": %.3f}\n", names[mode], N, ms * 1e3f / N );
		}
	}
	return 0;
}
