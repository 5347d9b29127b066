/* ref_softrast.cpp - TEST / BASELINE INFRASTRUCTURE: a thin extern "C" driver around the reference's
   CPU rasterizer (RenderCore_SoftRasterizer/rasterizer.cpp), compiled from the sources under
   /root/reference by oracle/Makefile.ref into oracle/_ref/libsoftrast_ref.so.  It times BASELINE
   config 1 (tinyapp + RenderCore_SoftRasterizer, 640x400, CPU) next to the MI355X core
   (tools/config1_plumbing.py).  No reference source is copied: this file fills the rasterizer's
   scene the way RenderCore_SoftRasterizer/rendercore.cpp does and calls Rasterizer::Render; only the
   OpenGL upload at the end of RenderCore::Render (rendercore.cpp:218-219) is left out (headless).
*/
#include "core_settings.h"   /* RenderCore_SoftRasterizer/core_settings.h (reference) */

#include <vector>

using namespace lh2core;

namespace
{
struct SoftRast
{
	Rasterizer rasterizer;
	Surface* target = nullptr;
	std::vector<Mesh*> meshes;
};
}

#define SR_API extern "C" __attribute__( (visibility( "default" )) )

/* RenderCore::Init + SetTarget (rendercore.cpp:27-57), one surface of exactly w x h */
SR_API void* sr_create( int w, int h )
{
	SoftRast* s = new SoftRast;
	s->rasterizer.Init();
	s->rasterizer.scene.root = new SGNode();
	s->target = new Surface();
	s->target->pixels = (uint*)MALLOC64( (size_t)w * h * sizeof( uint ) );
	s->target->width = w, s->target->height = h;
	s->rasterizer.Reinit( w, h, s->target );
	return s;
}

/* RenderCore::SetGeometry (rendercore.cpp:63-94): positions, bounds, connectivity, vertex normals,
   uvs, face normals and material ids from the CoreTri records */
SR_API int sr_set_geometry( void* h, int meshIdx, const float4* verts, int vertexCount, int triangleCount, const CoreTri* tri )
{
	SoftRast* s = (SoftRast*)h;
	if (vertexCount != 3 * triangleCount) return -1;
	Mesh* mesh;
	if (meshIdx >= (int)s->meshes.size()) s->meshes.push_back( mesh = new Mesh( vertexCount, triangleCount ) );
	else mesh = s->meshes[meshIdx];
	float3 bmin = make_float3( 1e34f ), bmax = -bmin;
	for (int i = 0; i < vertexCount; i++)
	{
		mesh->pos[i] = make_float3( verts[i] );
		bmin = fminf( bmin, mesh->pos[i] ), bmax = fmaxf( bmax, mesh->pos[i] );
	}
	mesh->bounds[0] = bmin, mesh->bounds[1] = bmax;
	for (int i = 0; i < triangleCount * 3; i++) mesh->tri[i] = i;
	for (int i = 0; i < triangleCount; i++)
	{
		const CoreTri& t = tri[i];
		mesh->norm[i * 3 + 0] = t.vN0, mesh->norm[i * 3 + 1] = t.vN1, mesh->norm[i * 3 + 2] = t.vN2;
		mesh->uv[i * 3 + 0] = make_float2( t.u0, t.v0 );
		mesh->uv[i * 3 + 1] = make_float2( t.u1, t.v1 );
		mesh->uv[i * 3 + 2] = make_float2( t.u2, t.v2 );
		mesh->N[i] = make_float3( t.Nx, t.Ny, t.Nz );
		mesh->material[i] = t.material;
	}
	return 0;
}

/* RenderCore::SetInstance (rendercore.cpp:100-121); meshIdx -1 truncates the instance list */
SR_API int sr_set_instance( void* h, int instanceIdx, int meshIdx, const float* m16 )
{
	SoftRast* s = (SoftRast*)h;
	std::vector<SGNode*>& child = s->rasterizer.scene.root->child;
	if (meshIdx == -1)
	{
		if ((int)child.size() > instanceIdx) child.resize( instanceIdx );
		return 0;
	}
	if (meshIdx >= (int)s->meshes.size() || instanceIdx > (int)child.size()) return -1;
	if (instanceIdx == (int)child.size()) child.push_back( s->meshes[meshIdx] );
	else child[instanceIdx] = s->meshes[meshIdx];
	mat4 M;
	for (int i = 0; i < 16; i++) M[i] = m16[i];
	child[instanceIdx]->localTransform = M;
	return 0;
}

/* RenderCore::SetTextures (rendercore.cpp:128-141): each texture's texels copied (pixelCount 32-bit texels,
   all MIP levels), its base size kept */
SR_API int sr_set_textures( void* h, const CoreTexDesc* tex, int count )
{
	SoftRast* s = (SoftRast*)h;
	std::vector<Texture*>& list = s->rasterizer.scene.texList;
	for (int i = 0; i < count; i++)
	{
		Texture* t;
		if (i < (int)list.size()) t = list[i];
		else list.push_back( t = new Texture() );
		t->pixels = (uint*)MALLOC64( tex[i].pixelCount * sizeof( uint ) );
		if (!tex[i].idata) return -1;
		memcpy( t->pixels, tex[i].idata, tex[i].pixelCount * sizeof( uint ) );
		t->width = tex[i].width, t->height = tex[i].height;
	}
	return 0;
}

/* RenderCore::SetMaterials (rendercore.cpp:147-172): the diffuse colour packed to 8 bits per channel, or the
   colour texture */
SR_API int sr_set_materials( void* h, const CoreMaterial* mat, int count )
{
	SoftRast* s = (SoftRast*)h;
	std::vector<Material*>& list = s->rasterizer.scene.matList;
	for (int i = 0; i < count; i++)
	{
		Material* m;
		if (i < (int)list.size()) m = list[i];
		else list.push_back( m = new Material() );
		m->texture = 0;
		const int texID = mat[i].color.textureID;
		if (texID == -1)
		{
			const float r = mat[i].color.value.x, g = mat[i].color.value.y, b = mat[i].color.value.z;
			m->diffuse = ((int)(b * 255.0f) << 16) + ((int)(g * 255.0f) << 8) + (int)(r * 255.0f);
		}
		else
		{
			if (texID >= (int)s->rasterizer.scene.texList.size()) return -1;
			m->texture = s->rasterizer.scene.texList[texID];
		}
	}
	return 0;
}

/* RenderCore::Render (rendercore.cpp:205-220) without the OpenGL texture upload */
SR_API void sr_render( void* h, const ViewPyramid* view )
{
	SoftRast* s = (SoftRast*)h;
	mat4 transform;
	const float3 X = normalize( view->p2 - view->p1 ), Y = normalize( view->p1 - view->p3 );
	const float3 Z = normalize( view->pos - 0.5f * (view->p2 + view->p3) );
	transform[0] = X.x, transform[4] = X.y, transform[8] = X.z;
	transform[1] = Y.x, transform[5] = Y.y, transform[9] = Y.z;
	transform[2] = Z.x, transform[6] = Z.y, transform[10] = Z.z;
	s->rasterizer.Render( mat4::Translate( view->pos ) * transform );
}

SR_API const uint* sr_pixels( void* h ) { return ((SoftRast*)h)->target->pixels; }
