/* multidevice.h - one render core spread over several HIP devices of one process (setting
   "deviceCount"), behind the unchanged CoreAPI_Base.

   SURVEY.md §8(e): the frame tile-partitions across the GPUs of a node and the accumulator is gathered
   once per frame.  An unchanged RenderSystem loads one core .so into one single-threaded process
   (lib/RenderSystem/core_api_base.cpp:97-132) and calls Render once per frame
   (rendersystem.cpp:228-238), so the partition lives inside the core: sub-core i renders the 8-row
   bands of rank i (RenderCore::SetTileBands, global pixel indices for RNG and blue noise, so the
   partition is exact) on device i, all sub-cores concurrently from one host thread each; then every
   sub-core's packed rows travel to device 0 by xGMI peer copy (hipMemcpyPeerAsync, peer access
   enabled) and are unpacked into device 0's accumulator, which is finalized for the display.  Scene
   and settings calls are broadcast.  With fewer physical devices than deviceCount the sub-cores
   share devices round-robin (a one-GPU box runs the same partition and gather, with local copies).
*/
#pragma once
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "rendercore.h"

namespace lh2 {

class MultiDevice
{
public:
	/* primary: the existing core (rank 0, on its device; not owned); count >= 2 sub-cores in total */
	MultiDevice( RenderCore* primary, int count );
	~MultiDevice();
	int Count() const { return (int)cores.size(); }
	RenderCore* Primary() { return cores[0]; }

	/* CoreAPI_Base, broadcast (scene, settings) or partitioned (target, render) */
	void SetProbePos( int x, int y );
	void SetTarget( uint32_t w, uint32_t h, uint32_t spp, uint32_t glTexture );
	void Setting( const char* name, float value );
	void Render( const lh2_ViewPyramid& view, int converge );
	void SetTextures( const lh2_CoreTexDesc* tex, int n );
	void SetMaterials( const lh2_CoreMaterial* mat, int n );
	void SetLights( const lh2_CoreLightTri* a, int na, const lh2_CorePointLight* p, int np, const lh2_CoreSpotLight* s, int ns,
		const lh2_CoreDirectionalLight* d, int nd );
	void SetSkyData( const float* px, uint32_t w, uint32_t h );
	void SetGeometry( int meshIdx, const float* v, int vc, int tc, const lh2_CoreTri* t, const uint32_t* alpha );
	void SetInstance( int idx, int mesh, const float* m16 );
	void UpdateToplevel();
	lh2_CoreStats GetCoreStats();
	/* extensions: the frame's totals over the sub-cores; device 0 holds the gathered accumulator */
	void GetRayCounts( uint32_t* out17 );
	void Synchronize();
	/* the settings the primary already has, onto the sub-cores created with this object */
	void ReplaySettings( const std::vector<std::pair<std::string, float>>& kv );

	static constexpr int band = 8;   /* rows per band, dealt round-robin over the sub-cores */
	/* settings the multi-device core keeps itself (not broadcast); false: not one of them */
	bool OwnSetting( const char* name, float value );

private:
	/* run f(i) for every sub-core i, each on its own worker thread with its device current */
	void ForEach( const std::function<void( int )>& f );
	void Worker( int i );
	void EnsureExchange();

	std::vector<RenderCore*> cores;           /* cores[0]: the primary */
	std::vector<int> devices;
	/* exchange buffers, double-buffered by frame parity: send[p][i] on device i (rank i's packed rows of a
	   frame of parity p), recv[i] on device 0.  copied[p][i] (device 0's stream, after its copy out of
	   send[p][i]) orders the pack of frame f + 2 into the same buffer after the copy of frame f: the host
	   queues frames ahead of the GPU, and a rank may finish frame f + 1 before device 0 gathers frame f */
	std::vector<void*> send[2], recv;
	std::vector<size_t> rowsOf;
	std::vector<hipEvent_t> packed, copied[2];
	std::vector<char> copyPending[2];
	int parity = 0;
	/* broadcast settings as last applied: a repeated value (RenderSystem sends six per frame,
	   rendersystem.cpp:231-236) costs no round trip over the worker threads */
	std::vector<std::pair<std::string, float>> applied;
	float gatherStallUs = 0;   /* debug: device 0 idles this long before each gather (tests of the ordering) */
	size_t exchangeBytes = 0;
	uint32_t width = 0, height = 0;
	/* worker pool */
	std::vector<std::thread> threads;
	std::mutex mtx;
	std::condition_variable cvWork, cvDone;
	const std::function<void( int )>* job = nullptr;
	int generation = 0, pending = 0;
	bool quit = false;
	std::vector<std::string> errors;
};

}  // namespace lh2
