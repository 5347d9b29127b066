/* ref_pins.cpp - TEST INFRASTRUCTURE: C entry points onto three host-side conversions of the reference,
   compiled from the reference sources where they lie (oracle/Makefile.ref -> oracle/_ref/libref_pins.so),
   so tests/test_golden.py can pin this repository's restatements to them bit for bit:

     pin_mat4_inverted   lighthouse2::mat4::Inverted (RenderSystem/common_types.h:586-628, header code):
                         the instance inverse that UpdateToplevel feeds the traversal
                         (RenderCore_OptixPrime_B/rendercore.cpp:481-505);
     pin_float_to_half   half_float::half( float ) (half2.1.0/half.hpp, HALF_ROUND_STYLE 1 = round to
                         nearest), the material colour conversion of RenderCore_OptixPrime_B
                         (core_settings.h:97-99, rendercore.cpp:353-399);
     pin_camera_view     Camera::GetView (RenderSystem/camera.cpp:96-117, with CalculateMatrix :40-58):
                         the ViewPyramid RenderSystem hands RenderCore::Render every frame.

   Nothing here is product code and nothing of the reference is copied: camera.cpp is compiled as it
   lies, and only the symbols reachable from these three functions survive --gc-sections. */
#include "platform.h"
#include "rendersystem.h"

#include <cstdint>
#include <cstring>
#include <new>

#define PIN_EXPORT extern "C" __attribute__( (visibility( "default" )) )

PIN_EXPORT void pin_mat4_inverted( const float* in16, float* out16 )
{
	mat4 m;
	std::memcpy( &m.cell[0], in16, 64 );
	const mat4 r = m.Inverted();
	std::memcpy( out16, &r.cell[0], 64 );
}

PIN_EXPORT void pin_float_to_half( const float* in, uint16_t* out, int n )
{
	for (int i = 0; i < n; i++)
	{
		const half_float::half h( in[i] );
		std::memcpy( out + i, &h, 2 );
	}
}

/* out17: pos, p1, p2, p3 (12 floats), aperture, spreadAngle, imagePlane, focalDistance, distortion */
PIN_EXPORT void pin_camera_view( const float* pos3, const float* dir3, float fov, float aspect, float focal, float aperture,
	float distortion, int pixelsX, int pixelsY, float* out17 )
{
	/* Camera's destructor saves the camera to XML (camera.cpp: ~Camera -> Serialize, tinyxml2): the pin's
	   camera lives in static storage and is never destroyed */
	alignas( Camera ) static unsigned char store[sizeof( Camera )];
	Camera& cam = *new (store) Camera();
	cam.position = make_float3( pos3[0], pos3[1], pos3[2] );
	cam.direction = make_float3( dir3[0], dir3[1], dir3[2] );
	cam.FOV = fov, cam.aspectRatio = aspect, cam.focalDistance = focal, cam.aperture = aperture, cam.distortion = distortion;
	cam.pixelCount = make_int2( pixelsX, pixelsY );
	const ViewPyramid v = cam.GetView();
	static_assert( sizeof( ViewPyramid ) == 17 * 4, "ViewPyramid layout" );
	std::memcpy( out17, &v, sizeof( ViewPyramid ) );
}
