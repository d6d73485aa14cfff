"""Malformed OBJ / MTL corpus through the C++ loader (pgrt_obj_load, csrc/objloader.cpp).

The reference parser (APP/objloader.cpp:53-507) scans with strtok / sscanf into fixed buffers and
indexes its vertex arrays without bounds checks, so malformed input is undefined behaviour there.
The restatement keeps the reference's semantics on well-formed files (tests/test_abi.py) and must,
on anything else, either return a consistent scene or fail with PGRT_ERR_IO and a message -- never
read or write out of bounds.  tools/asan_check.sh runs this file (with test_abi, test_oracle,
test_golden and test_tiles_gloo) against the AddressSanitizer + UBSan build (`make asan`).
"""
import numpy as np
import pytest

from pgi_raytracing_amd.raytracer import PgrtError, load_obj

V4 = "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\nvt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\n"
MTL = "newmtl a\nKd 0.1 0.2 0.3\nNs 8\n"

CORPUS = {
    "empty": ("", None),
    "comments_only": ("# nothing\n\n   \n# more\n", None),
    "face_before_vertices": ("f 1/1/1 2/2/1 3/3/1\n" + V4, None),
    "index_out_of_range": (V4 + "g a\nf 1/1/1 2/2/1 9/3/1\n", None),
    "normal_out_of_range": (V4 + "g a\nf 1/1/1 2/2/1 3/3/7\n", None),
    "negative_indices": (V4 + "g a\nf -1/-1/-1 -2/-2/-1 -3/-3/-1\n", None),
    "zero_index": (V4 + "g a\nf 0/1/1 2/2/1 3/3/1\n", None),
    "huge_index": (V4 + "g a\nf 99999999999999999999/1/1 2/2/1 3/3/1\n", None),
    "int_min_index": (V4 + "g a\nf 2147483648/1/1 2/2/1 3/3/1\n", None),
    # strtoll saturates to LLONG_MIN here if the sign ever reaches it (the reference's %[0-9]
    # scan stops at the '-', so the token keeps the previous face's indices)
    "huge_negative_index": (V4 + "g a\nf -99999999999999999999/1/1 2/2/1 3/3/1\n", None),
    "huge_negative_first_face": (V4 + "g a\nf 1/1/1 -99999999999999999999/-99999999999999999999/1 3/3/1\n", None),
    "missing_normals": (V4 + "g a\nf 1/1 2/2 3/3\n", None),
    "double_slash": (V4 + "g a\nf 1//1 2//1 3//1\n", None),
    "bare_indices": (V4 + "g a\nf 1 2 3\n", None),
    "two_vertex_face": (V4 + "g a\nf 1/1/1 2/2/1\n", None),
    "lone_f": (V4 + "g a\nf\n", None),
    "five_vertex_face_first": (V4 + "g a\nf 1/1/1 2/2/1 3/3/1 4/4/1 1/1/1\n", None),
    "quad_then_pentagon": (V4 + "g a\nf 1/1/1 2/2/1 3/3/1 4/4/1\nf 1/1/1 2/2/1 3/3/1 4/4/1 1/1/1\n", None),
    "usemtl_without_group": ("mtllib m.mtl\n" + V4 + "usemtl a\nf 1/1/1 2/2/1 3/3/1\n", MTL),
    "groups_without_faces": (V4 + "g a\ng b\ng\ng c\n", None),
    "truncated_coordinates": ("v 1.0\nv\nvn 0 0\nvt\nv 1 2 3\nv 0 1\nvn 1\nvt 0.5\ng a\nf 1/1/1 2/1/1 3/1/1\n", None),
    "non_finite_coordinates": ("v nan 0 0\nv inf 0 0\nv -inf 1 0\nvn 0 0 0\nvt nan inf\ng a\nf 1/1/1 2/1/1 3/1/1\n", None),
    "crlf_lines": (V4.replace("\n", "\r\n") + "g a\r\nf 1/1/1 2/2/1 3/3/1\r\n", None),
    "very_long_line": (V4 + "g " + "x" * 100000 + "\nf 1/1/1 2/2/1 3/3/1\n", None),
    "long_face_line": (V4 + "g a\nf " + " ".join(["1/1/1"] * 5000) + "\n", None),
    "missing_mtllib": ("mtllib nosuch.mtl\n" + V4 + "g a\nusemtl a\nf 1/1/1 2/2/1 3/3/1\n", None),
    "mtllib_without_name": ("mtllib\n" + V4 + "g a\nf 1/1/1 2/2/1 3/3/1\n", None),
    "malformed_mtl": ("mtllib m.mtl\n" + V4 + "g a\nusemtl \nf 1/1/1 2/2/1 3/3/1\n",
                      "newmtl\nKd garbage\nKs 1.0. 1.0\nNs\nshader x\nNi\nmap_Kd\nnewmtl b\nmap_Kd nosuch.png\n"),
    "binary_garbage": ("v \x01\x02\x03\nf \xff\xfe\n\x00\x00\ng \x7f\n", None),
}


@pytest.mark.parametrize("name", sorted(CORPUS))
def test_malformed_obj_is_rejected_or_consistent(tmp_path, name):
    obj, mtl = CORPUS[name]
    (tmp_path / "s.obj").write_bytes(obj.encode("latin-1"))
    if mtl is not None:
        (tmp_path / "m.mtl").write_bytes(mtl.encode("latin-1"))
    try:
        sc = load_obj(str(tmp_path / "s.obj"))
    except PgrtError as e:
        assert str(e)  # a message, not a crash
        return
    n = sc.num_triangles
    assert sc.positions.size == 9 * n and sc.normals.size == 9 * n and sc.uvs.size == 6 * n
    assert sc.material_ids.size == n
    assert ((sc.material_ids >= 0) & (sc.material_ids < len(sc.materials))).all()
    assert sum(s[2] for s in sc.surfaces) == n


def test_out_of_range_faces_fail_loudly(tmp_path):
    """An index past the vertex arrays (undefined behaviour in the reference) is an error here."""
    (tmp_path / "s.obj").write_text(CORPUS["index_out_of_range"][0])
    with pytest.raises(PgrtError, match="out of range"):
        load_obj(str(tmp_path / "s.obj"))


def test_well_formed_corpus_entries_load(tmp_path):
    (tmp_path / "s.obj").write_text(CORPUS["quad_then_pentagon"][0])
    sc = load_obj(str(tmp_path / "s.obj"))
    # the quad splits into two triangles; the pentagon line re-uses the quad's tokens (4 spaces
    # counted after trimming? no: 5 tokens -> neither 3 nor 4 spaces -> the previous tokens)
    assert sc.num_triangles == 3
    assert np.isfinite(sc.positions).all()
