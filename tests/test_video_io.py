"""CPU: the H.264 I_PCM .mp4 writer/reader (video_io.py) — the reference's mp4 output format
(inference.py:151-171, imaginaire/visualize/video.py) and .mp4 input (video2world.py:150-233).

No ffmpeg/decoder ships in this image, so the checks are structural: the ISO-BMFF box tree and
sample table, the SPS/PPS/slice syntax read back field by field, emulation-prevention-free PCM
payload, and an exact write -> read round trip of the Y'CbCr samples (parity of the colour
conversion to ffmpeg's is unpinned: no reference fixture holds decoded frames)."""
import struct

import numpy as np
import pytest

from cosmos_predict2 import video_io as vio


def _boxes(data, start, end):
    return {k: (s, e) for k, s, e in vio._boxes(data, start, end)}


@pytest.mark.parametrize("T,H,W", [(3, 36, 50), (2, 32, 48), (1, 17, 31)])
def test_mp4_round_trip(tmp_path, T, H, W):
    rng = np.random.RandomState(T * 100 + H)
    frames = rng.randint(0, 256, size=(T, H, W, 3), dtype=np.uint8)
    path = vio.write_mp4(frames, tmp_path / "v.mp4", fps=16)
    out = vio.read_mp4(path)
    He, We = H - H % 2, W - W % 2
    assert out.shape == (T, He, We, 3)
    # exactly the 4:2:0 samples that were written (edge-replicated to whole macroblocks, cropped back)
    Hp, Wp = -(-He // 16) * 16, -(-We // 16) * 16
    src = np.pad(frames[:, :He, :We], ((0, 0), (0, Hp - He), (0, Wp - We), (0, 0)), mode="edge")
    expect = vio.yuv420_to_rgb(*vio.rgb_to_yuv420(src))[:, :He, :We]
    assert np.array_equal(out, expect)


def test_mp4_smooth_image_fidelity(tmp_path):
    yy, xx = np.mgrid[0:64, 0:96]
    img = np.stack([(xx * 255 // 95), (yy * 255 // 63), ((xx + yy) * 255 // 158)], -1).astype(np.uint8)
    out = vio.read_mp4(vio.write_mp4(img[None].repeat(2, 0), tmp_path / "s.mp4"))
    err = np.abs(out.astype(int) - img[None].astype(int))
    assert err.mean() < 2.0 and err.max() <= 12


def test_mp4_structure(tmp_path):
    T, H, W = 4, 40, 64
    frames = np.full((T, H, W, 3), 128, np.uint8)
    data = open(vio.write_mp4(frames, tmp_path / "g.mp4", fps=16), "rb").read()
    top = _boxes(data, 0, len(data))
    assert list(top) == [b"ftyp", b"mdat", b"moov"]
    s, e = top[b"ftyp"]
    assert data[s:s + 4] == b"isom"
    stbl = vio._find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"minf", b"stbl"])
    assert set(_boxes(data, *stbl)) == {b"stsd", b"stts", b"stsc", b"stsz", b"stco"}
    s, _ = vio._find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"mdhd"])
    assert struct.unpack(">II", data[s + 12:s + 20]) == (16, T)  # timescale = fps, one tick per frame
    s, _ = vio._find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"hdlr"])
    assert data[s + 8:s + 12] == b"vide"
    s, _ = vio._find(data, *stbl, [b"stsz"])
    sizes = struct.unpack(">%dI" % T, data[s + 12:s + 12 + 4 * T])
    s, _ = vio._find(data, *stbl, [b"stco"])
    off = struct.unpack(">I", data[s + 8:s + 12])[0]
    assert off == top[b"mdat"][0] and sum(sizes) == top[b"mdat"][1] - top[b"mdat"][0]
    # every sample: one length-prefixed IDR NAL, nal_ref_idc 3
    for t, n in enumerate(sizes):
        smp = data[off:off + n]
        off += n
        assert struct.unpack(">I", smp[:4])[0] == n - 4 and smp[4] == 0x65
        pcm = np.frombuffer(smp, np.uint8)
        assert not ((pcm[:-2] == 0) & (pcm[1:-1] == 0) & (pcm[2:] <= 3)).any()  # no start-code emulation
        r = vio._Reader(vio._unescape(smp[4:]), 8)
        assert (r.ue(), r.ue(), r.ue(), r.u(4), r.ue()) == (0, 7, 0, 0, t & 1)  # I slice, IDR id alternates


def test_sps_pps_fields():
    sps = vio._unescape(vio._sps(5, 3, 14, 6))
    r = vio._Reader(sps, 0)
    assert r.u(8) == 0x67 and r.u(8) == 66 and r.u(8) == 0xC0 and r.u(8) == 51
    assert [r.ue() for _ in range(4)] == [0, 0, 2, 1]
    assert r.u(1) == 0 and r.ue() == 4 and r.ue() == 2 and r.u(1) == 1 and r.u(1) == 1
    assert r.u(1) == 1 and [r.ue() for _ in range(4)] == [0, 7, 0, 3]
    assert r.u(1) == 0 and r.u(1) == 1  # no VUI, stop bit
    pps = vio._pps()
    r = vio._Reader(pps, 0)
    assert r.u(8) == 0x68 and r.ue() == 0 and r.ue() == 0 and r.u(1) == 0  # CAVLC


def test_exp_golomb_and_escape():
    b = vio._Bits()
    for v in (0, 1, 2, 25, 300):
        b.ue(v)
    for v in (0, 1, -1, 7, -8):
        b.se(v)
    b.trailing()
    r = vio._Reader(b.tobytes())
    assert [r.ue() for _ in range(5)] == [0, 1, 2, 25, 300]
    assert [r.se() for _ in range(5)] == [0, 1, -1, 7, -8]
    raw = bytes([0, 0, 1, 5, 0, 0, 0, 0, 3, 0, 0])
    esc = vio._escape(raw)
    assert esc == bytes([0, 0, 3, 1, 5, 0, 0, 3, 0, 0, 3, 3, 0, 0])
    assert vio._unescape(esc) == raw


def test_mp4_rejects_bad_input(tmp_path):
    with pytest.raises(ValueError):
        vio.write_mp4(np.zeros((2, 8, 8), np.uint8), tmp_path / "x.mp4")
    with pytest.raises(ValueError):
        vio.write_mp4(np.zeros((0, 8, 8, 3), np.uint8), tmp_path / "x.mp4")
