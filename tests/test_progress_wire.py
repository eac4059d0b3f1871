"""lib.rs:128-138 ProgressMessage on the wire (postcard 0.7.3 + COBS, as discovery_app writes and
discovery_host_receiver reads): the C encoder against an independent Python restatement of the
postcard / COBS specifications and hand-derived known answers; decode round trips."""
import struct

import numpy as np
import pytest


def varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def cobs(data):  # COBS (Cheshire & Baker 1999), frame delimiter appended by to_vec_cobs
    out, block = bytearray(), bytearray()
    for b in data:
        if b == 0:
            out += bytes([len(block) + 1]) + block
            block = bytearray()
        else:
            block.append(b)
            if len(block) == 254:
                out += bytes([255]) + block
                block = bytearray()
    out += bytes([len(block) + 1]) + block
    return bytes(out) + b"\x00"


def postcard_msg(kind, w=0, h=0, spp=0, px=None):
    raw = varint(kind)
    if kind == 0:
        raw += varint(w) + varint(h) + varint(spp)
    elif kind == 1:
        raw += varint(px[0]) + varint(px[1]) + struct.pack("<3f", *px[2])
    return cobs(raw)


def test_known_answers(rtw):
    # ImageStart{32, 32, 50} (discovery_app raytracer.rs:55-66): postcard 00 20 20 32 -> COBS 01 04 20 20 32 | 00
    assert rtw.progress_encode(rtw.MSG_IMAGE_START, 32, 32, 50) == bytes([0x01, 0x04, 0x20, 0x20, 0x32, 0x00])
    assert rtw.progress_encode(rtw.MSG_IMAGE_END) == bytes([0x02, 0x02, 0x00])
    # Pixel{row 300, column 0, color (1, 0, -2)}: tag 01, varint 300 = AC 02, 00, 3 x f32 LE
    want = cobs(bytes([0x01, 0xAC, 0x02, 0x00]) + struct.pack("<3f", 1.0, 0.0, -2.0))
    assert rtw.progress_encode(rtw.MSG_PIXEL, pixel=(300, 0, (1.0, 0.0, -2.0))) == want
    assert want == bytes([0x04, 0x01, 0xAC, 0x02, 0x01, 0x01, 0x03, 0x80, 0x3F, 0x01, 0x01, 0x01, 0x01,
                          0x01, 0x01, 0x02, 0xC0, 0x00])


def test_random_messages_match_restatement_and_round_trip(rtw):
    rng = np.random.default_rng(1)
    for _ in range(500):
        kind = int(rng.integers(0, 3))
        if kind == 0:
            w, h, s = (int(x) for x in rng.integers(0, 2 ** 32, 3, dtype=np.uint64))
            frame = rtw.progress_encode(0, w, h, s)
            assert frame == postcard_msg(0, w, h, s)
            assert rtw.progress_decode(frame) == {"kind": 0, "width": w, "height": h, "samples_per_pixel": s}
        elif kind == 1:
            row, col = (int(x) for x in rng.integers(0, 1 << int(rng.integers(1, 33)), 2, dtype=np.uint64))
            color = rng.choice([0.0, -0.0, 1.5, 1e-40, np.inf], 3) if rng.uniform() < 0.3 else rng.normal(0, 50, 3)
            color = [float(np.float32(c)) for c in color]
            frame = rtw.progress_encode(1, pixel=(row, col, color))
            assert frame == postcard_msg(1, px=(row, col, color))
            d = rtw.progress_decode(frame)
            assert (d["row"], d["column"]) == (row, col)
            assert np.array_equal(np.float32(d["color"]).view(np.uint32), np.float32(color).view(np.uint32))
        else:
            assert rtw.progress_decode(rtw.progress_encode(2)) == {"kind": 2}
        assert frame[-1:] == b"\x00" and 0 not in frame[:-1]


def test_decode_errors_like_postcard(rtw):
    with pytest.raises(rtw.RtwError):  # DeserializeUnexpectedEnd: the 4 sync zeros give empty chunks
        rtw.progress_decode(b"")
    with pytest.raises(rtw.RtwError):
        rtw.progress_decode(bytes([0x02, 0x07, 0x00]))  # unknown enum tag
    with pytest.raises(rtw.RtwError):
        rtw.progress_decode(bytes([0x03, 0x01, 0x20, 0x00]))  # truncated Pixel
