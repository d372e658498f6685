"""Minimal PLY reader for point clouds (replaces the Open3D read used by the
reference at lib/utils.py:48 and scripts/pairwise_demo.py:75).  Supports
binary_little_endian / binary_big_endian / ascii vertex elements; returns the
x, y, z properties as float32 [N, 3] (Open3D widens them to float64)."""
import numpy as np

_TYPES = {"char": "i1", "uchar": "u1", "short": "i2", "ushort": "u2", "int": "i4", "uint": "u4", "float": "f4",
          "double": "f8", "int8": "i1", "uint8": "u1", "int16": "i2", "uint16": "u2", "int32": "i4",
          "uint32": "u4", "float32": "f4", "float64": "f8"}


def read_ply_xyz(path):
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError("%s: not a PLY file" % path)
        fmt, props, count, in_vertex, pre = None, [], 0, False, []
        while True:
            line = f.readline()
            if not line:
                raise ValueError("%s: truncated header" % path)
            tok = line.decode("ascii", "replace").split()
            if not tok:
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                in_vertex = tok[1] == "vertex"
                if in_vertex:
                    count = int(tok[2])
                elif count == 0:
                    pre.append((tok[1], int(tok[2])))
            elif tok[0] == "property" and in_vertex:
                if tok[1] == "list":
                    raise ValueError("list properties in the vertex element are not supported")
                props.append((tok[2], _TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        if pre:
            raise ValueError("elements before 'vertex' are not supported")
        if fmt == "ascii":
            data = np.loadtxt(f, max_rows=count, ndmin=2)
            names = [p[0] for p in props]
            return np.stack([data[:, names.index(a)] for a in "xyz"], 1).astype(np.float32)
        end = "<" if fmt == "binary_little_endian" else ">"
        dt = np.dtype([(n, end + t) for n, t in props])
        arr = np.frombuffer(f.read(dt.itemsize * count), dtype=dt, count=count)
        return np.stack([arr["x"], arr["y"], arr["z"]], 1).astype(np.float32)


def write_ply_xyz(path, xyz):
    xyz = np.asarray(xyz, dtype="<f4")
    with open(path, "wb") as f:
        f.write(("ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
                 "property float z\nend_header\n" % len(xyz)).encode())
        f.write(xyz.tobytes())
