"""Config 1's scene (BASELINE.json configs[0]: tinyapp's default scene) as a committed fixture.

Run in the container, where the reference assets are (they are not on the GPU box):
    python tools/make_config1_fixture.py  ->  tests/golden/config1_tinyapp.npz

tinyapp's PrepareScene (apps/tinyapp/main.cpp:34-45):
    AddScene( "scene.gltf", "data/pica/" )                 the pica diorama: 170 meshes, 339 nodes, 28 materials
    SetNodeTransform( "RootNode (gltf orientation matrix)", mat4::RotateX( -PI / 2 ) )
    AddMesh( "legocar.obj", "data/", 10.0f )                the car, vertices scaled by 10 at load
    AddMaterial( (100, 100, 80) ), AddQuad( (0, -1, 0), (0, 26, 0), 6.9, 6.9 )   the light, one instance
    AddInstance( car )                                      (the main loop then places it with
                                                            RotateY( 2r ) RotateZ( 0.2 sin 8r ) Translate( 0, 5, 0 ), r = 0 first)
The fixture keeps the loaders' inputs in compact form (numpy, no parsing at test time):
  * glTF primitives exactly as HostMesh::ConvertFromGTLFMesh reads them (host_mesh.cpp:310-469): indices,
    POSITION, NORMAL, TEXCOORD_0 (TANGENT is skipped by the reference), the material index;
  * the node hierarchy flattened into instances (mesh, world matrix), the root node's transform replaced by
    RotateX(-pi/2) as PrepareScene does;
  * glTF materials' baseColorFactor / metallicFactor / roughnessFactor and baseColorTexture index
    (HostMaterial::ConvertFrom, host_material.cpp:77-103);
  * the glTF textures in HostScene::AddScene's order (host_scene.cpp:260-271: one HostTexture per glTF texture,
    from its image): the image files' own bytes (lossless PNG; decoded at load by scene.tinyapp_scene with PIL to
    8-bit RGBA, as tinygltf's stb_image decode with req_comp 4 gives them, tiny_gltf.h:2202-2286).  One of the six
    images, Wax_Pastel_Label_02_baseColor.png, is missing from the reference (.MISSING_LARGE_BLOBS; the reference
    itself would stop at loading the glTF): its slot holds no bytes and the loader substitutes a documented
    stand-in texel block (scene.MISSING_TEXTURE_RGBA);
  * the OBJ's polygon soup after LoadGeometryFromOBJ's scale (host_mesh.cpp:131-305): positions (x 10), the
    per-corner normal indices and normals, per-face material; the .mtl Kd colours; tinyobjloader's default
    shininess 1 gives roughness min(1 - 1, 1) = 0 (host_material.cpp:41).
lighthouse2_amd/scene.py:tinyapp_scene() turns it into CoreTri records with the reference's conversions.
"""
from __future__ import annotations

import json
import math
import pathlib
import struct

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
REF = pathlib.Path("/root/reference/apps/tinyapp/data")
OUT = ROOT / "tests" / "golden" / "config1_tinyapp.npz"

COMP = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16, 5125: np.uint32, 5126: np.float32}
NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4, "MAT4": 16}


def accessor(g, buf, i):
    a = g["accessors"][i]
    v = g["bufferViews"][a["bufferView"]]
    dt = np.dtype(COMP[a["componentType"]])
    n, k = a["count"], NCOMP[a["type"]]
    stride = v.get("byteStride", dt.itemsize * k)
    off = v.get("byteOffset", 0) + a.get("byteOffset", 0)
    raw = np.frombuffer(buf, np.uint8, count=stride * (n - 1) + dt.itemsize * k, offset=off)
    if stride == dt.itemsize * k:
        return raw.view(dt).reshape(n, k) if k > 1 else raw.view(dt)
    return np.stack([raw[j * stride:j * stride + dt.itemsize * k].view(dt) for j in range(n)])


def rotate_x(a: float) -> np.ndarray:
    """mat4::RotateX (RenderSystem/common_types.h), row-major, float32 trig."""
    c, s = np.float32(math.cos(a)), np.float32(math.sin(a))
    m = np.eye(4, dtype=np.float32)
    m[1, 1], m[1, 2], m[2, 1], m[2, 2] = c, -s, s, c
    return m


def node_local(n) -> np.ndarray:
    """A glTF node's local matrix, row-major (glTF stores column-major; TRS = T * R * S)."""
    if "matrix" in n:
        return np.asarray(n["matrix"], np.float64).reshape(4, 4).T
    T = np.eye(4)
    if "translation" in n:
        T[:3, 3] = n["translation"]
    R = np.eye(4)
    if "rotation" in n:
        x, y, z, w = n["rotation"]
        R[:3, :3] = [[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]]
    S = np.eye(4)
    if "scale" in n:
        S[0, 0], S[1, 1], S[2, 2] = n["scale"]
    return T @ R @ S


def load_pica():
    g = json.load(open(REF / "pica" / "scene.gltf"))
    buf = (REF / "pica" / g["buffers"][0]["uri"]).read_bytes()
    # primitives of every mesh (ConvertFromGTLFMesh order)
    pos, nrm, uv, idx = [], [], [], []
    prim_mesh, prim_mat, prim_v, prim_i = [], [], [], []
    vb = ib = 0
    for mi, m in enumerate(g["meshes"]):
        for p in m["primitives"]:
            assert p.get("mode", 4) == 4, "only triangle lists in pica"
            ind = accessor(g, buf, p["indices"]).astype(np.int64).ravel()
            P = accessor(g, buf, p["attributes"]["POSITION"]).astype(np.float32)
            N = accessor(g, buf, p["attributes"]["NORMAL"]).astype(np.float32) if "NORMAL" in p["attributes"] else np.zeros((0, 3), np.float32)
            U = accessor(g, buf, p["attributes"]["TEXCOORD_0"]).astype(np.float32) if "TEXCOORD_0" in p["attributes"] else np.zeros((0, 2), np.float32)
            assert len(N) in (0, len(P)) and len(U) in (0, len(P))
            if len(N) == 0 or len(U) == 0:
                raise SystemExit("pica primitive without normals / uvs: extend the fixture format")
            pos.append(P), nrm.append(N), uv.append(U), idx.append(ind.astype(np.int32))
            prim_mesh.append(mi), prim_mat.append(p.get("material", 0))
            prim_v.append((vb, len(P))), prim_i.append((ib, len(ind)))
            vb += len(P)
            ib += len(ind)
    # instances: every node with a mesh, world = parent chain (HostNode: combined = parent * local), the
    # "RootNode (gltf orientation matrix)" node's transform set to RotateX(-pi/2) by PrepareScene
    world_of = {}
    inst_mesh, inst_T = [], []

    def visit(ni, parent):
        n = g["nodes"][ni]
        local = rotate_x(-math.pi / 2).astype(np.float64) if n.get("name") == "RootNode (gltf orientation matrix)" else node_local(n)
        W = parent @ local
        world_of[ni] = W
        if "mesh" in n:
            inst_mesh.append(n["mesh"]), inst_T.append(W.astype(np.float32))
        for c in n.get("children", []):
            visit(c, W)

    for r in g["scenes"][g.get("scene", 0)]["nodes"]:
        visit(r, np.eye(4))
    mats = g["materials"]
    color = np.array([m.get("pbrMetallicRoughness", {}).get("baseColorFactor", [1, 1, 1, 1])[:3] for m in mats], np.float32)
    metal = np.array([m.get("pbrMetallicRoughness", {}).get("metallicFactor", np.nan) for m in mats], np.float32)
    rough = np.array([m.get("pbrMetallicRoughness", {}).get("roughnessFactor", np.nan) for m in mats], np.float32)
    tex = np.array([m.get("pbrMetallicRoughness", {}).get("baseColorTexture", {}).get("index", -1) for m in mats], np.int32)
    # the textures (AddScene order), each the bytes of its image file (empty: missing from the reference)
    tex_png, tex_names = [], []
    for t in g.get("textures", []):
        uri = g["images"][t["source"]]["uri"]
        f = REF / "pica" / uri
        tex_png.append(np.frombuffer(f.read_bytes(), np.uint8) if f.exists() else np.zeros(0, np.uint8))
        tex_names.append(uri)
    png = {f"pica_tex_png_{i}": b for i, b in enumerate(tex_png)}
    return dict(pica_pos=np.concatenate(pos), pica_nrm=np.concatenate(nrm), pica_uv=np.concatenate(uv), pica_idx=np.concatenate(idx),
                pica_prim_mesh=np.array(prim_mesh, np.int32), pica_prim_mat=np.array(prim_mat, np.int32),
                pica_prim_v=np.array(prim_v, np.int64), pica_prim_i=np.array(prim_i, np.int64), pica_meshes=np.int32(len(g["meshes"])),
                pica_inst_mesh=np.array(inst_mesh, np.int32), pica_inst_T=np.array(inst_T, np.float32),
                pica_mat_color=color, pica_mat_metallic=metal, pica_mat_roughness=rough, pica_mat_tex=tex,
                pica_mat_names=np.array([m.get("name", "") for m in mats]), pica_tex_count=np.int32(len(tex_png)),
                pica_tex_names=np.array(tex_names), **png)


def load_car(scale: float = 10.0):
    """legocar.obj as tinyobjloader hands it to LoadGeometryFromOBJ: vertices, normals, faces (triangles; the
    file's faces are all triangles), per-face material (usemtl), the .mtl Kd colours."""
    v, vn, faces, fmat = [], [], [], []
    mtl_names, cur = [], -1
    for line in open(REF / "legocar.obj"):
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            v.append([float(x) for x in t[1:4]])
        elif t[0] == "vn":
            vn.append([float(x) for x in t[1:4]])
        elif t[0] == "usemtl":
            if t[1] not in mtl_names:
                mtl_names.append(t[1])
            cur = mtl_names.index(t[1])
        elif t[0] == "f":
            corners = [c.split("/") for c in t[1:]]
            assert len(corners) == 3, "legocar faces are triangles"
            faces.append([(int(c[0]) - 1, int(c[2]) - 1) for c in corners])
            fmat.append(cur)
    # tinyobjloader orders materials as the .mtl file lists them; usemtl indexes into that list
    kd, names = {}, []
    name = None
    for line in open(REF / "legocar.mtl"):
        t = line.split()
        if not t:
            continue
        if t[0] == "newmtl":
            name = t[1]
            names.append(name)
        elif t[0] == "Kd":
            kd[name] = [float(x) for x in t[1:4]]
    fmat = [names.index(mtl_names[m]) if m >= 0 else -1 for m in fmat]
    V = np.array(v, np.float32)
    # LoadGeometryFromOBJ: make_float4( v, 1 ) * transform, transform = mat4::Scale( scale ): x * s (+ 0 terms)
    V = (V * np.float32(scale)).astype(np.float32)
    F = np.array(faces, np.int32)       # (T, 3, 2): vertex index, normal index
    return dict(car_pos=V, car_nrm=np.array(vn, np.float32), car_face_v=F[:, :, 0], car_face_n=F[:, :, 1],
                car_face_mat=np.array(fmat, np.int32), car_mat_color=np.array([kd[n] for n in names], np.float32),
                car_mat_names=np.array(names))


def main():
    d = {}
    d.update(load_pica())
    d.update(load_car())
    OUT.parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(OUT, **d)
    print(f"{OUT}: {OUT.stat().st_size / 1e6:.2f} MB, pica {len(d['pica_idx']) // 3} tris in {len(d['pica_prim_mesh'])} primitives, "
          f"{len(d['pica_inst_mesh'])} instances; car {len(d['car_face_v'])} tris")


if __name__ == "__main__":
    main()
