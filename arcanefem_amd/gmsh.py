"""Gmsh 4.1 (binary and ASCII) mesh reader.

Host-side I/O for the meshes the reference's tests run on (`meshes/msh/*.msh`,
header ``$MeshFormat 4.1 1 8``).  It reproduces what the reference gets from
Arcane's MSH reader and uses on the hot path:

* node unique ids = Gmsh node tags (1-based), which is what the golden result
  files key on (`femutils/FemUtils.cc:104-169`, ``checkNodeResultFile``);
* cells = the elements of the mesh dimension (3-node triangles in 2D, 4-node
  tetrahedra in 3D), node order as stored in the file;
* named groups from ``$PhysicalNames``: a face group (dimension-1 physical
  group, e.g. ``horizontal`` in `modules/poisson/inputs/sphere.3D.arc`) and a
  node group (dimension-0 physical group, e.g. ``topLeftCorner`` in
  `modules/poisson/inputs/perforatedSquare.pointDirichlet.2D.arc`).  The
  reference applies Dirichlet conditions to ``face_group.nodeGroup()``
  (`femutils/ArcaneFemFunctionsGpu.h:497-504`), so every group is exposed as
  the set of nodes of its elements.
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

# Gmsh element type -> number of nodes (types used by the reference meshes)
_NODES_PER_TYPE = {1: 2, 2: 3, 3: 4, 4: 4, 5: 8, 6: 6, 7: 5, 8: 3, 9: 6,
                   10: 9, 11: 10, 15: 1}
_TYPE_DIM = {1: 1, 2: 2, 3: 2, 4: 3, 5: 3, 6: 3, 7: 3, 8: 1, 9: 2, 10: 2,
             11: 3, 15: 0}


@dataclasses.dataclass
class GmshMesh:
    dim: int
    node_tags: np.ndarray        # int64 [n_nodes]   Gmsh tags (unique ids)
    coords: np.ndarray           # float64 [n_nodes, 3]
    cells: np.ndarray            # int32 [n_cells, nv]  0-based node indices
    groups: dict                 # name -> (dim, int32 sorted unique node indices)
    face_groups: dict = dataclasses.field(default_factory=dict)
    # name -> int32 [n_faces, dim] node indices of the group's boundary faces
    # (edges in 2D, triangles in 3D), as stored in the file

    @property
    def n_nodes(self) -> int:
        return int(self.node_tags.shape[0])

    @property
    def n_cells(self) -> int:
        return int(self.cells.shape[0])

    def group_faces(self, name: str) -> np.ndarray:
        if name not in self.face_groups:
            raise KeyError(f"no face group named {name!r}; have {sorted(self.face_groups)}")
        return self.face_groups[name]

    def face_cells(self, faces: np.ndarray) -> np.ndarray:
        """For each boundary face, the cell it bounds (Arcane's face->cell
        connectivity, which the reference uses to orient boundary normals)."""
        return boundary_face_cells(self.cells, faces)

    def group_nodes(self, name: str) -> np.ndarray:
        if name not in self.groups:
            raise KeyError(f"no physical group named {name!r}; have {sorted(self.groups)}")
        return self.groups[name][1]


class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        self.p = 0

    def line(self) -> str:
        e = self.d.index(b"\n", self.p)
        s = self.d[self.p:e].decode("latin-1").strip()
        self.p = e + 1
        return s

    def skip_ws(self):
        while self.p < len(self.d) and self.d[self.p:self.p + 1] in (b"\n", b"\r", b" ", b"\t"):
            self.p += 1

    def unpack(self, fmt: str):
        sz = struct.calcsize(fmt)
        v = struct.unpack_from(fmt, self.d, self.p)
        self.p += sz
        return v

    def array(self, dtype, count):
        a = np.frombuffer(self.d, dtype=dtype, count=count, offset=self.p)
        self.p += a.nbytes
        return a


def read_gmsh(path: str) -> GmshMesh:
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    binary = False
    phys_names = {}          # (dim, tag) -> name
    entity_phys = {}         # (dim, entity_tag) -> [phys tags]
    node_tag_list, coord_list = [], []
    elem_blocks = []         # (dim, entity_tag, type, conn ndarray[n, nn] of node tags)
    ascii_tokens = None

    def tok():
        nonlocal ascii_tokens
        return next(ascii_tokens)

    while r.p < len(data):
        r.skip_ws()
        if r.p >= len(data):
            break
        hdr = r.line()
        if hdr == "$MeshFormat":
            version, ftype, dsize = r.line().split()
            if not version.startswith("4.1"):
                raise ValueError(f"{path}: only Gmsh 4.1 is supported (got {version})")
            binary = ftype == "1"
            if binary:
                if int(dsize) != 8:
                    raise ValueError("size_t must be 8 bytes")
                (one,) = r.unpack("<i")
                if one != 1:
                    raise ValueError("big-endian Gmsh files are not supported")
            r.skip_ws()
            assert r.line() == "$EndMeshFormat"
        elif hdr == "$PhysicalNames":
            n = int(r.line())
            for _ in range(n):
                parts = r.line().split(maxsplit=2)
                phys_names[(int(parts[0]), int(parts[1]))] = parts[2].strip('"')
            assert r.line() == "$EndPhysicalNames"
        elif hdr == "$Entities":
            if binary:
                counts = r.unpack("<4Q")
                for dim in range(4):
                    for _ in range(counts[dim]):
                        (tag,) = r.unpack("<i")
                        r.unpack("<3d" if dim == 0 else "<6d")
                        (nphys,) = r.unpack("<Q")
                        phys = list(r.unpack(f"<{nphys}i")) if nphys else []
                        entity_phys[(dim, tag)] = phys
                        if dim > 0:
                            (nb,) = r.unpack("<Q")
                            r.unpack(f"<{nb}i")
                r.skip_ws()
                assert r.line() == "$EndEntities"
            else:
                counts = [int(x) for x in r.line().split()]
                for dim in range(4):
                    for _ in range(counts[dim]):
                        toks = r.line().split()
                        tag = int(toks[0])
                        off = 4 if dim == 0 else 7
                        nphys = int(toks[off])
                        entity_phys[(dim, tag)] = [int(x) for x in toks[off + 1: off + 1 + nphys]]
                assert r.line() == "$EndEntities"
        elif hdr == "$Nodes":
            if binary:
                nblocks, nnodes, _, _ = r.unpack("<4Q")
                for _ in range(nblocks):
                    edim, etag, parametric = r.unpack("<3i")
                    (nb,) = r.unpack("<Q")
                    tags = r.array("<u8", nb).astype(np.int64)
                    ncomp = 3 + (edim if parametric else 0)
                    xyz = r.array("<f8", nb * ncomp).reshape(nb, ncomp)[:, :3]
                    node_tag_list.append(tags)
                    coord_list.append(np.array(xyz))
                r.skip_ws()
                assert r.line() == "$EndNodes"
            else:
                nblocks, nnodes, _, _ = (int(x) for x in r.line().split())
                for _ in range(nblocks):
                    edim, etag, parametric, nb = (int(x) for x in r.line().split())
                    tags = np.array([int(r.line()) for _ in range(nb)], dtype=np.int64)
                    xyz = np.array([[float(v) for v in r.line().split()[:3]] for _ in range(nb)]).reshape(nb, 3)
                    node_tag_list.append(tags)
                    coord_list.append(xyz)
                assert r.line() == "$EndNodes"
        elif hdr == "$Elements":
            if binary:
                nblocks, nelem, _, _ = r.unpack("<4Q")
                for _ in range(nblocks):
                    edim, etag, etype = r.unpack("<3i")
                    (nb,) = r.unpack("<Q")
                    nn = _NODES_PER_TYPE[etype]
                    raw = r.array("<u8", nb * (nn + 1)).reshape(nb, nn + 1)
                    elem_blocks.append((edim, etag, etype, raw[:, 1:].astype(np.int64)))
                r.skip_ws()
                assert r.line() == "$EndElements"
            else:
                nblocks, nelem, _, _ = (int(x) for x in r.line().split())
                for _ in range(nblocks):
                    edim, etag, etype, nb = (int(x) for x in r.line().split())
                    rows = [[int(x) for x in r.line().split()] for _ in range(nb)]
                    elem_blocks.append((edim, etag, etype, np.array(rows, dtype=np.int64)[:, 1:]))
                assert r.line() == "$EndElements"
        else:
            # skip unknown section
            end = "$End" + hdr[1:]
            idx = data.index(end.encode(), r.p)
            r.p = idx + len(end)

    node_tags = np.concatenate(node_tag_list)
    coords = np.concatenate(coord_list).astype(np.float64)
    order = np.argsort(node_tags, kind="stable")
    node_tags = node_tags[order]
    coords = coords[order]
    max_tag = int(node_tags.max())
    tag_to_idx = np.full(max_tag + 1, -1, dtype=np.int64)
    tag_to_idx[node_tags] = np.arange(node_tags.shape[0])

    mesh_dim = max(_TYPE_DIM[b[2]] for b in elem_blocks)
    cell_blocks = [b for b in elem_blocks if _TYPE_DIM[b[2]] == mesh_dim]
    types = {b[2] for b in cell_blocks}
    if types - {2, 4}:
        raise ValueError(f"{path}: only P1 triangles/tetrahedra are supported as cells (got types {types})")
    cells = np.concatenate([tag_to_idx[b[3]] for b in cell_blocks]).astype(np.int32)

    groups_acc: dict = {}
    for edim, etag, etype, conn in elem_blocks:
        for ptag in entity_phys.get((edim, etag), []):
            name = phys_names.get((edim, ptag))
            if name is None:
                continue
            groups_acc.setdefault(name, (edim, []))[1].append(tag_to_idx[conn].ravel())
    groups = {name: (gd, np.unique(np.concatenate(lst)).astype(np.int32))
              for name, (gd, lst) in groups_acc.items()}
    faces_acc: dict = {}
    for edim, etag, etype, conn in elem_blocks:
        if edim != mesh_dim - 1 or _NODES_PER_TYPE[etype] != mesh_dim:
            continue
        for ptag in entity_phys.get((edim, etag), []):
            name = phys_names.get((edim, ptag))
            if name is not None:
                faces_acc.setdefault(name, []).append(tag_to_idx[conn])
    face_groups = {name: np.concatenate(lst).astype(np.int32) for name, lst in faces_acc.items()}
    return GmshMesh(dim=mesh_dim, node_tags=node_tags, coords=coords, cells=cells, groups=groups,
                    face_groups=face_groups)


def boundary_face_cells(cells: np.ndarray, faces: np.ndarray) -> np.ndarray:
    """Cell owning each face (the faces of a P1 simplex are its nv choose dim
    node subsets); -1 when no cell has the face."""
    cells = np.asarray(cells)
    nv = cells.shape[1]
    dim = nv - 1
    lookup = {}
    for a in range(nv):
        sub = np.sort(np.delete(cells, a, axis=1), axis=1)
        for c, key in enumerate(map(tuple, sub)):
            lookup.setdefault(key, c)
    fs = np.sort(np.asarray(faces).reshape(-1, dim), axis=1)
    return np.array([lookup.get(tuple(f), -1) for f in fs], dtype=np.int32)


def read_node_result_file(path: str) -> dict:
    """Golden file format `uid value [value...]` (`femutils/FemUtils.cc:122-135`)."""
    out = {}
    with open(path) as f:
        for line in f:
            parts = line.split()
            if not parts:
                continue
            vals = [float(x) for x in parts[1:]]
            out[int(parts[0])] = vals[0] if len(vals) == 1 else np.array(vals)
    return out
