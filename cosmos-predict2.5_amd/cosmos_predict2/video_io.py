"""MP4 video output (and input of the files it writes) without ffmpeg.

The reference writes its results as H.264 .mp4 at 16 fps (cosmos_predict2/inference.py:151-171 via
imaginaire/visualize/video.py:45-…, imageio + ffmpeg) and reads .mp4 inputs with a decoder library
(video2world.py:150-233). Neither library ships in this image, so this module writes a standard
H.264 stream whose every macroblock is I_PCM — the uncompressed intra macroblock type every baseline
decoder supports (ITU-T H.264 §7.3.5, mb_type 25 in I slices) — inside an ISO-BMFF container
(`ftyp` / `mdat` / `moov` with an `avc1` + `avcC` sample entry). The files play in ordinary players;
they are large (1.5 bytes per pixel, 4:2:0) because nothing is compressed. `read_mp4` decodes exactly
this subset (I_PCM-only baseline streams, as written here) so Video2World can take such a file back
as its input; other H.264 streams raise.

Colour: RGB -> Y'CbCr BT.601 limited range, 2x2 chroma averaging (ffmpeg's default for yuv420p).
"""
from __future__ import annotations

import struct
from pathlib import Path
from typing import List, Tuple

import numpy as np

_PROFILE_BASELINE = 66
_LEVEL = 51
_MB_HDR = bytes([0x0D, 0x00])  # ue(25) = 0000 11010 + pcm alignment zero bits, when byte aligned


# ----------------------------------------------------------------------------- bit writer / reader
class _Bits:
    def __init__(self):
        self.bits: List[int] = []

    def u(self, n: int, v: int) -> None:
        self.bits.extend((v >> (n - 1 - i)) & 1 for i in range(n))

    def ue(self, v: int) -> None:
        x = v + 1
        n = x.bit_length()
        self.u(n - 1, 0)
        self.u(n, x)

    def se(self, v: int) -> None:
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def align_zero(self) -> None:
        while len(self.bits) % 8:
            self.bits.append(0)

    def trailing(self) -> None:  # rbsp_trailing_bits
        self.bits.append(1)
        self.align_zero()

    def tobytes(self) -> bytes:
        assert len(self.bits) % 8 == 0
        return np.packbits(np.array(self.bits, dtype=np.uint8)).tobytes()


class _Reader:
    def __init__(self, data: bytes, pos_bits: int = 0):
        self.data = data
        self.pos = pos_bits

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            byte = self.data[self.pos >> 3]
            v = (v << 1) | ((byte >> (7 - (self.pos & 7))) & 1)
            self.pos += 1
        return v

    def ue(self) -> int:
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + self.u(z)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)

    def align(self) -> None:
        self.pos = (self.pos + 7) & ~7


def _start_code_like(a: np.ndarray, last_max: int) -> np.ndarray:
    """Positions i + 2 where a[i] == a[i+1] == 0 and a[i+2] <= last_max."""
    if a.size < 3:
        return np.zeros(0, np.int64)
    return np.nonzero((a[:-2] == 0) & (a[1:-1] == 0) & (a[2:] <= last_max))[0] + 2


def _escape(rbsp: bytes) -> bytes:
    """Emulation prevention: 0x000000..03 -> 0x000003xx (H.264 §7.4.1)."""
    if _start_code_like(np.frombuffer(rbsp, np.uint8), 3).size == 0:
        return rbsp
    out = bytearray()
    zeros = 0
    for b in rbsp:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


def _unescape(ebsp: bytes) -> bytes:
    if _start_code_like(np.frombuffer(ebsp, np.uint8), 3).size == 0:
        return ebsp
    out = bytearray()
    zeros = 0
    i = 0
    while i < len(ebsp):
        b = ebsp[i]
        if zeros >= 2 and b == 3:
            zeros = 0
            i += 1
            continue
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
        i += 1
    return bytes(out)


# ----------------------------------------------------------------------------- colour
def rgb_to_yuv420(frames: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """uint8 [T, H, W, 3] (H, W even) -> Y [T, H, W], Cb/Cr [T, H/2, W/2], BT.601 limited range."""
    f = frames.astype(np.float32) / 255.0
    r, g, b = f[..., 0], f[..., 1], f[..., 2]
    y = 16.0 + 65.481 * r + 128.553 * g + 24.966 * b
    cb = 128.0 - 37.797 * r - 74.203 * g + 112.0 * b
    cr = 128.0 + 112.0 * r - 93.786 * g - 18.214 * b
    T, H, W = y.shape

    def sub(c):
        return c.reshape(T, H // 2, 2, W // 2, 2).mean(axis=(2, 4))

    q = lambda a: np.clip(np.rint(a), 1, 255).astype(np.uint8)  # noqa: E731 - PCM samples 1..255
    return q(y), q(sub(cb)), q(sub(cr))


def yuv420_to_rgb(y: np.ndarray, cb: np.ndarray, cr: np.ndarray) -> np.ndarray:
    """Inverse of rgb_to_yuv420 (nearest chroma upsampling) -> uint8 [T, H, W, 3]."""
    yf = (y.astype(np.float32) - 16.0) * (255.0 / 219.0)
    cbf = np.repeat(np.repeat(cb.astype(np.float32) - 128.0, 2, axis=1), 2, axis=2) * (255.0 / 224.0)
    crf = np.repeat(np.repeat(cr.astype(np.float32) - 128.0, 2, axis=1), 2, axis=2) * (255.0 / 224.0)
    r = yf + 1.402 * crf
    g = yf - 0.344136 * cbf - 0.714136 * crf
    b = yf + 1.772 * cbf
    return np.clip(np.rint(np.stack([r, g, b], -1)), 0, 255).astype(np.uint8)


# ----------------------------------------------------------------------------- H.264 I_PCM stream
def _sps(w_mbs: int, h_mbs: int, crop_r: int, crop_b: int) -> bytes:
    b = _Bits()
    b.u(8, 0x67)                      # nal_ref_idc 3, nal_unit_type 7 (SPS)
    b.u(8, _PROFILE_BASELINE)
    b.u(8, 0xC0)                      # constraint_set0/1 (baseline-compatible)
    b.u(8, _LEVEL)
    b.ue(0)                           # seq_parameter_set_id
    b.ue(0)                           # log2_max_frame_num_minus4
    b.ue(2)                           # pic_order_cnt_type 2: output order = decode order
    b.ue(1)                           # max_num_ref_frames
    b.u(1, 0)                         # gaps_in_frame_num_value_allowed_flag
    b.ue(w_mbs - 1)
    b.ue(h_mbs - 1)
    b.u(1, 1)                         # frame_mbs_only_flag
    b.u(1, 1)                         # direct_8x8_inference_flag
    if crop_r or crop_b:
        b.u(1, 1)                     # frame_cropping_flag; offsets in 2-pixel units (4:2:0 frames)
        b.ue(0)
        b.ue(crop_r // 2)
        b.ue(0)
        b.ue(crop_b // 2)
    else:
        b.u(1, 0)
    b.u(1, 0)                         # vui_parameters_present_flag
    b.trailing()
    return _escape(b.tobytes())


def _pps() -> bytes:
    b = _Bits()
    b.u(8, 0x68)                      # nal_ref_idc 3, nal_unit_type 8 (PPS)
    b.ue(0)                           # pic_parameter_set_id
    b.ue(0)                           # seq_parameter_set_id
    b.u(1, 0)                         # entropy_coding_mode_flag: CAVLC
    b.u(1, 0)                         # bottom_field_pic_order_in_frame_present_flag
    b.ue(0)                           # num_slice_groups_minus1
    b.ue(0)
    b.ue(0)                           # num_ref_idx_l0/l1_default_active_minus1
    b.u(1, 0)
    b.u(2, 0)                         # weighted_pred_flag, weighted_bipred_idc
    b.se(0)
    b.se(0)
    b.se(0)                           # pic_init_qp/qs_minus26, chroma_qp_index_offset
    b.u(1, 1)                         # deblocking_filter_control_present_flag
    b.u(1, 0)                         # constrained_intra_pred_flag
    b.u(1, 0)                         # redundant_pic_cnt_present_flag
    b.trailing()
    return _escape(b.tobytes())


def _idr_slice(mbs: np.ndarray, idr_pic_id: int) -> bytes:
    """One IDR picture as a single I slice of I_PCM macroblocks. mbs: uint8 [n_mb, 384] (256 luma
    raster, 64 Cb, 64 Cr), samples >= 1 so the PCM bytes never form a start-code prefix."""
    b = _Bits()
    b.u(8, 0x65)                      # nal_ref_idc 3, nal_unit_type 5 (IDR slice)
    b.ue(0)                           # first_mb_in_slice
    b.ue(7)                           # slice_type 7: I (all slices of the picture)
    b.ue(0)                           # pic_parameter_set_id
    b.u(4, 0)                         # frame_num (log2_max_frame_num 4)
    b.ue(idr_pic_id)
    b.u(1, 0)
    b.u(1, 0)                         # dec_ref_pic_marking: no_output_of_prior_pics, long_term_reference
    b.se(0)                           # slice_qp_delta
    b.ue(1)                           # disable_deblocking_filter_idc 1 (PCM needs no deblocking)
    b.ue(25)                          # mb_type I_PCM of macroblock 0
    b.align_zero()                    # pcm_alignment_zero_bits
    head = _escape(b.tobytes())
    body = np.empty((mbs.shape[0], 386), np.uint8)
    body[:, :2] = np.frombuffer(_MB_HDR, np.uint8)
    body[:, 2:] = mbs
    # macroblock 0's mb_type is in `head`; every later one is the byte-aligned 0x0D 0x00
    flat = body.reshape(-1)[2:]
    z = flat == 0
    if (z[:-1] & z[1:]).any():  # cannot happen with samples >= 1; escape the general way if it does
        return head + _escape(flat.tobytes() + b"\x80")
    return head + flat.tobytes() + b"\x80"  # rbsp_slice_trailing_bits


def _macroblocks(y: np.ndarray, cb: np.ndarray, cr: np.ndarray) -> np.ndarray:
    H, W = y.shape
    hm, wm = H // 16, W // 16
    ly = y.reshape(hm, 16, wm, 16).transpose(0, 2, 1, 3).reshape(hm * wm, 256)
    lb = cb.reshape(hm, 8, wm, 8).transpose(0, 2, 1, 3).reshape(hm * wm, 64)
    lr = cr.reshape(hm, 8, wm, 8).transpose(0, 2, 1, 3).reshape(hm * wm, 64)
    return np.concatenate([ly, lb, lr], axis=1)


# ----------------------------------------------------------------------------- ISO BMFF
def _box(kind: bytes, *payload: bytes) -> bytes:
    data = b"".join(payload)
    return struct.pack(">I", 8 + len(data)) + kind + data


def _full(kind: bytes, version: int, flags: int, *payload: bytes) -> bytes:
    return _box(kind, struct.pack(">I", (version << 24) | flags), *payload)


_MATRIX = struct.pack(">9i", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


def write_mp4(frames: np.ndarray, path, fps: int = 16) -> str:
    """uint8 [T, H, W, 3] RGB -> H.264 (I_PCM) .mp4 at `fps`. Returns the path written."""
    frames = np.asarray(frames)
    if frames.dtype != np.uint8 or frames.ndim != 4 or frames.shape[-1] != 3:
        raise ValueError("write_mp4 expects uint8 frames [T, H, W, 3]")
    T, H, W, _ = frames.shape
    if T == 0 or H < 2 or W < 2:
        raise ValueError(f"empty or too small video {frames.shape}")
    # even dimensions for 4:2:0 (a trailing odd row/column is dropped), padded to whole macroblocks
    # by edge replication and cropped back in the SPS
    He, We = H - H % 2, W - W % 2
    Hp, Wp = -(-He // 16) * 16, -(-We // 16) * 16
    sps, pps = _sps(Wp // 16, Hp // 16, Wp - We, Hp - He), _pps()
    samples = []
    for t in range(T):
        src = np.pad(frames[t:t + 1, :He, :We], ((0, 0), (0, Hp - He), (0, Wp - We), (0, 0)), mode="edge")
        y, cb, cr = rgb_to_yuv420(src)
        nal = _idr_slice(_macroblocks(y[0], cb[0], cr[0]), t & 1)
        samples.append(struct.pack(">I", len(nal)) + nal)
    avcc = _box(b"avcC", bytes([1, _PROFILE_BASELINE, 0xC0, _LEVEL, 0xFF, 0xE1]), struct.pack(">H", len(sps)), sps,
                bytes([1]), struct.pack(">H", len(pps)), pps)
    name = b"cosmos-predict2.5 I_PCM"
    avc1 = _box(b"avc1", bytes(6), struct.pack(">H", 1), bytes(16), struct.pack(">HH", We, He),
                struct.pack(">II", 0x480000, 0x480000), bytes(4), struct.pack(">H", 1),
                bytes([len(name)]) + name + bytes(31 - len(name)), struct.pack(">hh", 0x18, -1), avcc)
    ftyp = _box(b"ftyp", b"isom", struct.pack(">I", 0x200), b"isomiso2avc1mp41")
    mdat_payload = b"".join(samples)
    if len(ftyp) + 8 + len(mdat_payload) >= 1 << 32:
        raise ValueError("video too large for a 32-bit mp4 (chunk offsets)")
    chunk_off = len(ftyp) + 8
    dur_ms = int(round(1000 * T / fps))
    stbl = _box(b"stbl",
                _full(b"stsd", 0, 0, struct.pack(">I", 1), avc1),
                _full(b"stts", 0, 0, struct.pack(">III", 1, T, 1)),
                _full(b"stsc", 0, 0, struct.pack(">IIII", 1, 1, T, 1)),
                _full(b"stsz", 0, 0, struct.pack(">II", 0, T), b"".join(struct.pack(">I", len(s)) for s in samples)),
                _full(b"stco", 0, 0, struct.pack(">II", 1, chunk_off)))
    minf = _box(b"minf", _full(b"vmhd", 0, 1, bytes(8)),
                _box(b"dinf", _full(b"dref", 0, 0, struct.pack(">I", 1), _full(b"url ", 0, 1))), stbl)
    mdia = _box(b"mdia", _full(b"mdhd", 0, 0, struct.pack(">IIIIHH", 0, 0, fps, T, 0x55C4, 0)),
                _full(b"hdlr", 0, 0, bytes(4), b"vide", bytes(12), b"VideoHandler\x00"), minf)
    tkhd = _full(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, 1, 0, dur_ms), bytes(8),
                 struct.pack(">hhhH", 0, 0, 0, 0), _MATRIX, struct.pack(">II", We << 16, He << 16))
    mvhd = _full(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, 1000, dur_ms), struct.pack(">IH", 0x10000, 0x100),
                 bytes(10), _MATRIX, bytes(24), struct.pack(">I", 2))
    moov = _box(b"moov", mvhd, _box(b"trak", tkhd, mdia))
    path = str(path)
    with open(path, "wb") as f:
        f.write(ftyp)
        f.write(struct.pack(">I", 8 + len(mdat_payload)) + b"mdat")
        f.write(mdat_payload)
        f.write(moov)
    return path


# ----------------------------------------------------------------------------- reader (this subset)
def _boxes(data: bytes, start: int, end: int):
    i = start
    while i + 8 <= end:
        size, kind = struct.unpack(">I4s", data[i:i + 8])
        hdr = 8
        if size == 1:
            size = struct.unpack(">Q", data[i + 8:i + 16])[0]
            hdr = 16
        elif size == 0:
            size = end - i
        yield kind, i + hdr, i + size
        i += size


def _find(data: bytes, start: int, end: int, path: List[bytes]) -> Tuple[int, int]:
    for kind, s, e in _boxes(data, start, end):
        if kind == path[0]:
            return (s, e) if len(path) == 1 else _find(data, s, e, path[1:])
    raise ValueError(f"mp4: box {path[0].decode()} not found")


def read_mp4(path) -> np.ndarray:
    """Decode an I_PCM-only H.264 .mp4 (as written by write_mp4) -> uint8 RGB [T, H, W, 3]."""
    data = Path(path).read_bytes()
    stbl = _find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"minf", b"stbl"])
    s, e = _find(data, *stbl, [b"stsd"])
    avc1 = s + 8  # full-box header + entry_count
    if data[avc1 + 4:avc1 + 8] != b"avc1":
        raise ValueError("mp4: not an H.264 (avc1) track")
    s, e = _find(data, avc1 + 8 + 78, avc1 + struct.unpack(">I", data[avc1:avc1 + 4])[0], [b"avcC"])
    sps_len = struct.unpack(">H", data[s + 6:s + 8])[0]
    sps = _unescape(data[s + 8:s + 8 + sps_len])
    r = _Reader(sps, 8)
    if r.u(8) != _PROFILE_BASELINE:
        raise ValueError("mp4: only the baseline I_PCM streams written by write_mp4 are readable here")
    r.u(16)
    r.ue(), r.ue()
    if r.ue() != 2:
        raise ValueError("mp4: unsupported pic_order_cnt_type")
    r.ue(), r.u(1)
    wm, hm = r.ue() + 1, r.ue() + 1
    r.u(1), r.u(1)
    crop = [0, 0, 0, 0]
    if r.u(1):
        crop = [2 * r.ue() for _ in range(4)]
    s, e = _find(data, *stbl, [b"stsz"])
    n = struct.unpack(">I", data[s + 8:s + 12])[0]
    sizes = struct.unpack(">%dI" % n, data[s + 12:s + 12 + 4 * n])
    s, e = _find(data, *stbl, [b"stco"])
    off = struct.unpack(">I", data[s + 8:s + 12])[0]
    Hp, Wp = 16 * hm, 16 * wm
    ys = np.empty((n, Hp, Wp), np.uint8)
    cbs = np.empty((n, Hp // 2, Wp // 2), np.uint8)
    crs = np.empty((n, Hp // 2, Wp // 2), np.uint8)
    for t, size in enumerate(sizes):
        sample = data[off:off + size]
        off += size
        nal_len = struct.unpack(">I", sample[:4])[0]
        nal = _unescape(sample[4:4 + nal_len])
        r = _Reader(nal, 8)
        r.ue()
        if r.ue() % 5 != 2:
            raise ValueError("mp4: not an I slice")
        r.ue(), r.u(4), r.ue(), r.u(1), r.u(1), r.se()
        if r.ue() != 1:
            raise ValueError("mp4: unexpected deblocking mode")
        nmb = wm * hm
        mbs = np.empty((nmb, 384), np.uint8)
        if r.ue() != 25:
            raise ValueError("mp4: only I_PCM macroblocks are supported")
        r.align()
        p = r.pos >> 3
        mbs[0] = np.frombuffer(nal, np.uint8, 384, p)
        # every later macroblock starts byte aligned: ue(25) + alignment = 0x0D 0x00, then 384 samples
        rest = np.frombuffer(nal, np.uint8, (nmb - 1) * 386, p + 384).reshape(nmb - 1, 386)
        if nmb > 1 and not ((rest[:, 0] == 0x0D).all() and (rest[:, 1] == 0).all()):
            raise ValueError("mp4: only I_PCM macroblocks are supported")
        mbs[1:] = rest[:, 2:]
        ys[t] = mbs[:, :256].reshape(hm, wm, 16, 16).transpose(0, 2, 1, 3).reshape(Hp, Wp)
        cbs[t] = mbs[:, 256:320].reshape(hm, wm, 8, 8).transpose(0, 2, 1, 3).reshape(Hp // 2, Wp // 2)
        crs[t] = mbs[:, 320:].reshape(hm, wm, 8, 8).transpose(0, 2, 1, 3).reshape(Hp // 2, Wp // 2)
    rgb = yuv420_to_rgb(ys, cbs, crs)
    return rgb[:, crop[2]:Hp - crop[3], crop[0]:Wp - crop[1]]
