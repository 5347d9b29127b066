/* multidevice.cpp - the render core over several HIP devices of one process (multidevice.h). */
#include "multidevice.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace lh2 {

#define MD_CHK( stmt ) do { hipError_t e_ = (stmt); if (e_ != hipSuccess) FatalError( "%s failed: %s", #stmt, hipGetErrorString( e_ ) ); } while (0)

MultiDevice::MultiDevice( RenderCore* primary, int count )
{
	int physical = 0;
	MD_CHK( hipGetDeviceCount( &physical ) );
	const int d0 = primary->Device();
	cores.push_back( primary ), devices.push_back( d0 );
	for (int i = 1; i < count; i++)
	{
		const int d = (d0 + i) % std::max( 1, physical );
		MD_CHK( hipSetDevice( d ) );
		/* xGMI peer copies into device 0 (and a peer's reads of it) without staging */
		int can = 0;
		if (d != d0 && hipDeviceCanAccessPeer( &can, d, d0 ) == hipSuccess && can)
		{
			const hipError_t e = hipDeviceEnablePeerAccess( d0, 0 );
			if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) FatalError( "hipDeviceEnablePeerAccess: %s", hipGetErrorString( e ) );
			(void)hipGetLastError();
		}
		RenderCore* c = new RenderCore();
		c->Init();
		cores.push_back( c ), devices.push_back( d );
	}
	MD_CHK( hipSetDevice( d0 ) );
	for (int i = 1; i < count; i++)
	{
		int can = 0;
		if (devices[i] != d0 && hipDeviceCanAccessPeer( &can, d0, devices[i] ) == hipSuccess && can)
		{
			const hipError_t e = hipDeviceEnablePeerAccess( devices[i], 0 );
			if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) FatalError( "hipDeviceEnablePeerAccess: %s", hipGetErrorString( e ) );
			(void)hipGetLastError();
		}
	}
	for (int p = 0; p < 2; p++) send[p].assign( count, nullptr ), copied[p].assign( count, nullptr ), copyPending[p].assign( count, 0 );
	recv.assign( count, nullptr ), rowsOf.assign( count, 0 ), packed.assign( count, nullptr );
	errors.assign( count, std::string() );
	for (int i = 0; i < count; i++)
	{
		MD_CHK( hipSetDevice( devices[i] ) );
		MD_CHK( hipEventCreateWithFlags( &packed[i], hipEventDisableTiming ) );
	}
	MD_CHK( hipSetDevice( d0 ) );
	for (int p = 0; p < 2; p++) for (int i = 0; i < count; i++) MD_CHK( hipEventCreateWithFlags( &copied[p][i], hipEventDisableTiming ) );
	MD_CHK( hipSetDevice( d0 ) );
	for (int i = 0; i < count; i++) threads.emplace_back( &MultiDevice::Worker, this, i );
}

MultiDevice::~MultiDevice()
{
	{
		std::lock_guard<std::mutex> lk( mtx );
		quit = true;
	}
	cvWork.notify_all();
	for (auto& t : threads) t.join();
	for (int i = 0; i < Count(); i++)
	{
		(void)hipSetDevice( devices[i] );
		(void)hipDeviceSynchronize();
		for (int p = 0; p < 2; p++) if (send[p][i]) (void)hipFree( send[p][i] );
		if (packed[i]) (void)hipEventDestroy( packed[i] );
		(void)hipSetDevice( devices[0] );
		if (recv[i]) (void)hipFree( recv[i] );
		for (int p = 0; p < 2; p++) if (copied[p][i]) (void)hipEventDestroy( copied[p][i] );
		if (i > 0) { (void)hipSetDevice( devices[i] ); cores[i]->Shutdown(); delete cores[i]; }
	}
	(void)hipSetDevice( devices[0] );
}

/* ---- worker pool: one host thread per sub-core, its device current ---------------------- */
void MultiDevice::Worker( int i )
{
	(void)hipSetDevice( devices[i] );
	int seen = 0;
	while (true)
	{
		const std::function<void( int )>* f;
		{
			std::unique_lock<std::mutex> lk( mtx );
			cvWork.wait( lk, [&] { return quit || generation != seen; } );
			if (quit) return;
			seen = generation, f = job;
		}
		try { (*f)( i ); }
		catch (const std::exception& e) { errors[i] = e.what(); }
		catch (...) { errors[i] = "unknown error"; }
		{
			std::lock_guard<std::mutex> lk( mtx );
			if (--pending == 0) cvDone.notify_one();
		}
	}
}

void MultiDevice::ForEach( const std::function<void( int )>& f )
{
	{
		std::lock_guard<std::mutex> lk( mtx );
		job = &f, pending = Count(), generation++;
		for (auto& e : errors) e.clear();
	}
	cvWork.notify_all();
	{
		std::unique_lock<std::mutex> lk( mtx );
		cvDone.wait( lk, [&] { return pending == 0; } );
	}
	(void)hipSetDevice( devices[0] );   /* the caller's thread stays on device 0 */
	for (int i = 0; i < Count(); i++) if (!errors[i].empty()) throw std::runtime_error( "device " + std::to_string( devices[i] ) + ": " + errors[i] );
}

/* ---- broadcast calls ---------------------------------------------------------------------- */
void MultiDevice::SetProbePos( int x, int y ) { for (auto* c : cores) c->SetProbePos( x, y ); }
void MultiDevice::Setting( const char* name, float value )
{
	if (OwnSetting( name, value )) return;
	for (const auto& kv : applied) if (kv.first == name && kv.second == value) return;   /* unchanged: no round trip */
	ForEach( [&]( int i ) { cores[i]->Setting( name, value ); } );
	bool found = false;
	for (auto& kv : applied) if (kv.first == name) kv.second = value, found = true;
	if (!found) applied.emplace_back( name, value );
}
void MultiDevice::ReplaySettings( const std::vector<std::pair<std::string, float>>& kv )
{
	std::vector<std::pair<std::string, float>> bc;
	for (const auto& e : kv) if (!OwnSetting( e.first.c_str(), e.second )) bc.push_back( e );
	ForEach( [&]( int i ) { if (i > 0) for (const auto& e : bc) cores[i]->Setting( e.first.c_str(), e.second ); } );
	applied = bc;
}
bool MultiDevice::OwnSetting( const char* name, float value )
{
	if (!strcmp( name, "gatherStallUs" )) { gatherStallUs = std::max( 0.0f, value ); return true; }
	return false;
}
void MultiDevice::SetTextures( const lh2_CoreTexDesc* tex, int n ) { ForEach( [&]( int i ) { cores[i]->SetTextures( tex, n ); } ); }
void MultiDevice::SetMaterials( const lh2_CoreMaterial* mat, int n ) { ForEach( [&]( int i ) { cores[i]->SetMaterials( mat, n ); } ); }
void MultiDevice::SetLights( const lh2_CoreLightTri* a, int na, const lh2_CorePointLight* p, int np, const lh2_CoreSpotLight* s, int ns,
	const lh2_CoreDirectionalLight* d, int nd )
{
	ForEach( [&]( int i ) { cores[i]->SetLights( a, na, p, np, s, ns, d, nd ); } );
}
void MultiDevice::SetSkyData( const float* px, uint32_t w, uint32_t h ) { ForEach( [&]( int i ) { cores[i]->SetSkyData( px, w, h ); } ); }
/* one BLAS build per mesh, not one per device: core 0 takes the mesh (a CPU build is deferred), the other
   sub-cores upload its shading triangles and share core 0's deferred build (RenderCore::AdoptGeometry) */
void MultiDevice::SetGeometry( int meshIdx, const float* v, int vc, int tc, const lh2_CoreTri* t, const uint32_t* alpha )
{
	cores[0]->SetGeometry( meshIdx, v, vc, tc, t, alpha );
	ForEach( [&]( int i ) { if (i > 0) cores[i]->AdoptGeometry( meshIdx, tc, t, *cores[0] ); } );
}
void MultiDevice::SetInstance( int idx, int mesh, const float* m16 ) { ForEach( [&]( int i ) { cores[i]->SetInstance( idx, mesh, m16 ); } ); }
/* the shared builds run first, on core 0's thread pool (the host's threads once, not N pools); then every sub-core uploads
   them to its device and builds its TLAS */
void MultiDevice::UpdateToplevel()
{
	cores[0]->FlushPendingBuilds();
	ForEach( [&]( int i ) { cores[i]->UpdateToplevel(); } );
}

/* ---- partitioned calls ------------------------------------------------------------------- */
void MultiDevice::SetTarget( uint32_t w, uint32_t h, uint32_t spp, uint32_t glTexture )
{
	const int n = Count();
	ForEach( [&]( int i ) {
		cores[i]->SetTarget( w, h, spp );
		cores[i]->SetTileBands( i, n, band );
	} );
	cores[0]->SetInteropTexture( glTexture );   /* the display copy happens on device 0 after the gather */
	cores[0]->displayAtFinalize = true;         /* ... in FinalizeFrame only, not in its own Render */
	width = w, height = h;
	EnsureExchange();
}

void MultiDevice::EnsureExchange()
{
	const int n = Count();
	size_t maxRows = 0;
	for (int i = 0; i < n; i++)
	{
		size_t rows = 0;
		for (uint32_t y = (uint32_t)(i * band); y < height; y += (uint32_t)(n * band)) rows += std::min<uint32_t>( band, height - y );
		rowsOf[i] = rows, maxRows = std::max( maxRows, rows );
	}
	const size_t bytes = maxRows * width * sizeof( float4 );
	if (bytes <= exchangeBytes) return;
	Synchronize();   /* frames in flight may still read the old buffers */
	for (int i = 1; i < n; i++)
	{
		MD_CHK( hipSetDevice( devices[i] ) );
		for (int p = 0; p < 2; p++)
		{
			if (send[p][i]) MD_CHK( hipFree( send[p][i] ) );
			MD_CHK( hipMalloc( &send[p][i], bytes ) );
			copyPending[p][i] = 0;
		}
		MD_CHK( hipSetDevice( devices[0] ) );
		if (recv[i]) MD_CHK( hipFree( recv[i] ) );
		MD_CHK( hipMalloc( &recv[i], bytes ) );
	}
	MD_CHK( hipSetDevice( devices[0] ) );
	exchangeBytes = bytes;
}

void MultiDevice::Render( const lh2_ViewPyramid& view, int converge )
{
	const int n = Count(), p = parity;
	parity ^= 1;
	/* every device renders its bands; ranks > 0 pack them for the gather (async on their streams), into
	   this frame parity's send buffer once device 0 has copied the frame two back out of it */
	ForEach( [&]( int i ) {
		cores[i]->Render( view, converge );
		if (i > 0)
		{
			if (copyPending[p][i]) MD_CHK( hipStreamWaitEvent( cores[i]->Stream(), copied[p][i], 0 ) );
			cores[i]->PackTile( send[p][i] );
			MD_CHK( hipEventRecord( packed[i], cores[i]->Stream() ) );
		}
	} );
	/* the gather on device 0's stream: peer copy (xGMI DMA) of each rank's rows, then unpack */
	RenderCore* c0 = cores[0];
	if (gatherStallUs > 0) lh2_launch_spin( (uint64_t)(gatherStallUs * 100.0f), c0->Stream() );   /* 100 MHz ticks */
	for (int i = 1; i < n; i++)
	{
		MD_CHK( hipStreamWaitEvent( c0->Stream(), packed[i], 0 ) );
		const size_t bytes = rowsOf[i] * width * sizeof( float4 );
		if (devices[i] == devices[0]) MD_CHK( hipMemcpyAsync( recv[i], send[p][i], bytes, hipMemcpyDeviceToDevice, c0->Stream() ) );
		else MD_CHK( hipMemcpyPeerAsync( recv[i], devices[0], send[p][i], devices[i], bytes, c0->Stream() ) );
		MD_CHK( hipEventRecord( copied[p][i], c0->Stream() ) );
		copyPending[p][i] = 1;
		c0->UnpackTile( recv[i], i, n, band );
	}
	c0->FinalizeFrame();
}

void MultiDevice::Synchronize() { ForEach( [&]( int i ) { cores[i]->Synchronize(); } ); }

/* CoreStats of the frame: rays summed over the devices, times the slowest device's */
lh2_CoreStats MultiDevice::GetCoreStats()
{
	std::vector<lh2_CoreStats> st( Count() );
	ForEach( [&]( int i ) { st[i] = cores[i]->GetCoreStats(); } );
	lh2_CoreStats s = st[0];
	for (int i = 1; i < Count(); i++)
	{
		const lh2_CoreStats& t = st[i];
		s.totalRays += t.totalRays, s.totalExtensionRays += t.totalExtensionRays, s.totalShadowRays += t.totalShadowRays;
		s.primaryRayCount += t.primaryRayCount, s.bounce1RayCount += t.bounce1RayCount, s.deepRayCount += t.deepRayCount;
		s.renderTime = std::max( s.renderTime, t.renderTime ), s.traceTime0 = std::max( s.traceTime0, t.traceTime0 );
		s.traceTime1 = std::max( s.traceTime1, t.traceTime1 ), s.traceTimeX = std::max( s.traceTimeX, t.traceTimeX );
		s.shadowTraceTime = std::max( s.shadowTraceTime, t.shadowTraceTime ), s.shadeTime = std::max( s.shadeTime, t.shadeTime );
		s.bvhBuildTime = std::max( s.bvhBuildTime, t.bvhBuildTime );
		/* the probe pixel lies in exactly one device's bands */
		if (t.probedInstid != -1 || t.probedTriid != -1) s.probedInstid = t.probedInstid, s.probedTriid = t.probedTriid, s.probedDist = t.probedDist;
	}
	return s;
}

void MultiDevice::GetRayCounts( uint32_t* out17 )
{
	std::vector<uint32_t> all( 17 * (size_t)Count() );
	ForEach( [&]( int i ) { cores[i]->GetRayCounts( all.data() + 17 * (size_t)i ); } );
	for (int k = 0; k < 17; k++)
	{
		out17[k] = 0;
		for (int i = 0; i < Count(); i++) out17[k] += all[17 * (size_t)i + k];
	}
}

}  // namespace lh2
