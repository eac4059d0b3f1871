"""Decode the reference's image textures into binary PPM (P6) files this build loads.

The GPU box has no copy of /root/reference and the build ships no JPEG decoder, so
models/earthmap.jpg (ImageTexture::open in scenes.rs:256, :292, :567) is decoded here once, with
Pillow's libjpeg, into models/earthmap.ppm (RGB8, top row first, as image::open(..).to_rgb8()
hands it to image_texture.rs:23-30).  JPEG decoders may differ from the `image 0.25.2` crate's by
+-1 in a few pixels (IDCT / chroma upsampling rounding): parity unpinned at that boundary.

    python models/make_images.py [/root/reference/models]
"""
import sys
from pathlib import Path

from PIL import Image

src = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/models")
out = Path(__file__).resolve().parent
for stem in ("earthmap",):
    im = Image.open(src / f"{stem}.jpg").convert("RGB")
    w, h = im.size
    data = im.tobytes()
    (out / f"{stem}.ppm").write_bytes(b"P6\n%d %d\n255\n" % (w, h) + data)
    print(f"{stem}: {w}x{h} -> {out / (stem + '.ppm')}")
