"""Decode the scene textures once into raw "PGRTTEX1" sidecars (<file>.pgrttex) for C++ hosts
that have no image decoder (FreeImage is not available; texture.cpp:5-54 decoded with it).
Same bytes as pgi_raytracing_amd.scene.TextureData.from_file: BGR(A), top-down, pitch rounded
to 4 bytes like FreeImage_GetPitch; JPEGs decoded like FreeImage's JPEG_DEFAULT load (IFAST).
A sidecar older than its image or than the decoder library is rewritten."""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def convert(path: str) -> str:
    from pgi_raytracing_amd.scene import TextureData

    t = TextureData.from_file(path)
    out = path + ".pgrttex"
    with open(out, "wb") as f:
        f.write(b"PGRTTEX1")
        f.write(struct.pack("<4i", t.width, t.height, t.pitch, t.bpp))
        f.write(t.data.tobytes())
    return out


def convert_all() -> list:
    assets = os.path.join(ROOT, "assets")
    lib = os.path.join(ROOT, "pgi_raytracing_amd", "lib", "libpgrt_image.so")
    decoder_mtime = os.path.getmtime(lib) if os.path.exists(lib) else 0.0
    done = []
    for dirpath, _, files in os.walk(assets):
        for f in files:
            if f.lower().endswith((".jpg", ".jpeg", ".png")):
                p = os.path.join(dirpath, f)
                side = p + ".pgrttex"
                if (not os.path.exists(side) or os.path.getmtime(side) < os.path.getmtime(p)
                        or os.path.getmtime(side) < decoder_mtime):
                    done.append(convert(p))
    return done


if __name__ == "__main__":
    for p in sys.argv[1:] or []:
        print(convert(p))
    if len(sys.argv) == 1:
        print("\n".join(convert_all()))
