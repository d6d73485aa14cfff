"""Python restatement of LoadOBJ / LoadMTL (objloader.cpp:53-507) -- TEST INFRASTRUCTURE.

Used only by tests/ to check the product's C++ loader (pgrt_obj_load) quirk for quirk:
strtok line splitting (empty lines vanish), three passes, sscanf("%*s %f %f %f") partial
parses ("Ks 1.0. 1.0 1.0" -> only Ks.x is read), vn normalised in float32 (vector3.cpp:155-167),
'f' lines classified by their space count (3 -> triangle, 4 -> quad split (0,1,2)+(0,2,3),
anything else re-uses the previous face's tokens), "%[0-9]/%[0-9]/%[0-9]" index parsing whose
failed conversions keep the previous buffer contents, and the surface material = the last
usemtl seen when the NEXT 'g' line (or EOF) closes the group.
"""
from __future__ import annotations

import os
import re

import numpy as np

_FLOAT = re.compile(r"\s*([+-]?(?:(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?|inf(?:inity)?|nan))", re.I)


def _scan_floats(line: str, n: int, defaults):
    """sscanf(line, "%*s %f %f %f"): skip the first token, then read up to n floats; fields
    after the first failed conversion keep their previous value."""
    out = list(defaults)
    m = re.match(r"\s*\S+", line)
    if not m:
        return out
    pos = m.end()
    for i in range(n):
        fm = _FLOAT.match(line, pos)
        if not fm:
            break
        out[i] = float(np.float32(fm.group(1)))
        pos = fm.end()
    return out


def _scan_word(line: str):
    """sscanf(line, "%*s %s"): second whitespace-delimited token or None."""
    parts = line.split()
    return parts[1] if len(parts) >= 2 else None


def _lines(text: str):
    return [l for l in text.split("\n") if l != ""]


def _trim(s: str) -> str:
    return s.strip(" \t\n\v\f\r\0")


def _normalize(v):
    x, y, z = (np.float32(c) for c in v)
    norm = x * x + y * y + z * z
    if norm != 0:
        rn = np.float32(1) / np.sqrt(norm, dtype=np.float32)
        x, y, z = x * rn, y * rn, z * rn
    return [float(x), float(y), float(z)]


def load_mtl(file_name: str, path: str, materials: list):
    """LoadMTL (objloader.cpp:53-208).  Materials are dicts; textures are path strings."""
    with open(file_name, "r", newline="") as f:
        text = f.read()
    material = None
    material_name = ""
    for line in _lines(text):
        if line[0] == "#":
            continue
        if line.startswith("newmtl"):
            if material is not None:
                material["name"] = material_name
                if not any(m["name"] == material_name for m in materials):
                    materials.append(material)
            w = _scan_word(line)
            if w is not None:
                material_name = w
            material = dict(name="default", ambient=[0.1, 0.1, 0.1], diffuse=[0.4, 0.4, 0.4],
                            specular=[0.8, 0.8, 0.8], emission=[0.0, 0.0, 0.0], shininess=1.0,
                            ior=1.5, type=0, map_kd=None)
            continue
        tmp = _trim(line)
        if material is None:
            continue
        if tmp.startswith("Ka"):
            material["ambient"] = _scan_floats(tmp, 3, material["ambient"])
        if tmp.startswith("shader"):
            m = re.match(r"\s*\S+\s*([+-]?\d+)", tmp)
            if m:
                material["type"] = int(m.group(1))
        if tmp.startswith("Ni"):
            material["ior"] = _scan_floats(tmp, 1, [material["ior"]])[0]
        if tmp.startswith("Kd"):
            material["diffuse"] = _scan_floats(tmp, 3, material["diffuse"])
        if tmp.startswith("Ks"):
            material["specular"] = _scan_floats(tmp, 3, material["specular"])
        if tmp.startswith("Ke"):
            material["emission"] = _scan_floats(tmp, 3, material["emission"])
        if tmp.startswith("Ns"):
            material["shininess"] = _scan_floats(tmp, 1, [material["shininess"]])[0]
        if tmp.startswith("map_Kd"):
            w = _scan_word(tmp)
            if w is not None:
                material["map_kd"] = path + w
    if material is not None:
        material["name"] = material_name
        materials.append(material)


def load_obj(file_name: str, flip_yz: bool = False):
    """LoadOBJ (objloader.cpp:210-507).

    Returns (surfaces, materials); a surface is dict(name, material index or -1,
    positions (T,3,3), normals (T,3,3), uvs (T,3,2))."""
    with open(file_name, "r", newline="") as f:
        text = f.read()
    slash = file_name.rfind("/")
    path = file_name[: slash + 1] if slash >= 0 else ""
    lines = _lines(text)
    materials: list = []
    for line in lines:
        if line[0] == "m":
            w = _scan_word(line)
            if w is not None:
                load_mtl(path + w, path, materials)
    verts, norms, tcs = [], [], []
    for line in lines:
        if line[0] == "v" and len(line) > 1:
            if line[1] == " ":
                x, y, z = _scan_floats(line, 3, [0.0, 0.0, 0.0])
                verts.append([x, -z, y] if flip_yz else [x, y, z])
            elif line[1] == "n":
                x, y, z = _scan_floats(line, 3, [0.0, 0.0, 0.0])
                n = [x, -z, y] if flip_yz else [x, y, z]
                norms.append(_normalize(n))
            elif line[1] == "t":
                u, v, _ = _scan_floats(line, 3, [0.0, 0.0, 0.0])
                tcs.append([u, v])
    surfaces = []
    face = []
    group_name = ""
    material_name = ""
    tokens = ["", "", "", ""]  # char vertices_indices[4][26], persistent
    idx_buf = ["", "", ""]     # char vertex_indices[3][8], persistent

    def close_group():
        mi = -1
        for i, m in enumerate(materials):
            if m["name"] == material_name:
                mi = i
                break
        f = np.asarray(face, dtype=object)
        T = len(face) // 3
        pos = np.array([fv[0] for fv in face], np.float32).reshape(T, 3, 3)
        nrm = np.array([fv[1] for fv in face], np.float32).reshape(T, 3, 3)
        uv = np.array([fv[2] for fv in face], np.float32).reshape(T, 3, 2)
        surfaces.append(dict(name=group_name, material=mi, positions=pos, normals=nrm, uvs=uv))
        del f

    def parse_vertex(tok):
        # sscanf(tok, "%[0-9]/%[0-9]/%[0-9]", ...): stops at the first failed conversion
        pos = 0
        for k in range(3):
            m = re.match(r"[0-9]+", tok[pos:])
            if not m:
                break
            idx_buf[k] = m.group(0)
            pos += m.end()
            if k < 2:
                if pos < len(tok) and tok[pos] == "/":
                    pos += 1
                else:
                    break
        vi, ti, ni = (int(idx_buf[k]) - 1 if idx_buf[k] else -1 for k in range(3))
        return (verts[vi], norms[ni], tcs[ti])

    for line in lines:
        c = line[0]
        if c == "g":
            if face:
                close_group()
                face = []
            w = _scan_word(line)
            if w is not None:
                group_name = w
        elif c == "u":
            w = _scan_word(line)
            if w is not None:
                material_name = w
        elif c == "f":
            t = line.rstrip(" \t\n\v\f\r")
            no_spaces = t.count(" ")
            parts = t.split()
            if no_spaces == 3:
                tokens[0:3] = parts[1:4]
            elif no_spaces == 4:
                tokens[0:4] = parts[1:5]
            for i in range(3):
                face.append(parse_vertex(tokens[i]))
            if no_spaces == 4:
                for i in (0, 2, 3):
                    face.append(parse_vertex(tokens[i]))
    if face:
        close_group()
    return surfaces, materials
