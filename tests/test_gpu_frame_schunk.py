"""GPU tier: contiguous frames opened through the reference's own entry points
(blosc2_schunk_from_buffer, blosc/schunk.c:731-750; blosc2_schunk_open / _open_offset, 366-470;
frame_to_schunk, blosc/frame.c:2941-3245) against the reference build (oracle/_ref) opening the same
frames: the frames written by the reference (tests/golden/frame_*.b2frame) and frames the reference
writes here with metalayers and vlmetalayers (blosc2_meta_add / blosc2_vlmeta_add, then
blosc2_schunk_to_buffer).

Expected: the same super-chunk fields and counters for both flavours (copy and frame-attached),
byte-identical chunks (special offsets become the same 32-byte special chunks), the same
decompressed chunks and slices, and the same (vl)metalayer names and contents.  data_len is the
index's allocation size, an implementation detail (the reference leaves it 0 for a frame).
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, HERE)

import blosc2_amd as B  # noqa: E402

pytestmark = pytest.mark.gpu

GOLD = os.path.join(HERE, "golden")
FRAMES = sorted(f[:-8] for f in os.listdir(GOLD) if f.endswith(".b2frame"))
FIELDS = ("nchunks", "current_nchunk", "nbytes", "cbytes", "chunksize", "flags2", "typesize", "blocksize",
          "clevel", "compcode", "compcode_meta", "splitmode", "use_dict", "nmetalayers", "nvlmetalayers")


class Meta(C.Structure):
    """blosc2_metalayer (reference include/blosc2.h:1810-1814)."""
    _fields_ = [("name", C.c_char_p), ("content", C.POINTER(C.c_uint8)), ("content_len", C.c_int32)]


def _ref():
    from oracle_lib import ref
    R = ref()
    if R is None:
        pytest.skip("reference build absent")
    return B.bind_schunk(R)


def _fields(sc):
    s = sc.s
    d = {k: getattr(s, k) for k in FIELDS}
    d["filters"] = list(s.filters)
    d["filters_meta"] = list(s.filters_meta)
    d["contiguous"] = bool(s.storage.contents.contiguous)
    d["urlpath"] = s.storage.contents.urlpath
    return d


def _layers(sc, vl):
    s = sc.s
    n, arr = (s.nvlmetalayers, s.vlmetalayers) if vl else (s.nmetalayers, s.metalayers)
    out = []
    for i in range(n):
        m = C.cast(arr[i], C.POINTER(Meta)).contents
        out.append((m.name, bytes(np.ctypeslib.as_array(m.content, (m.content_len,))) if m.content_len else b""))
    return out


def _same(a, b):
    assert _fields(a) == _fields(b), (_fields(a), _fields(b))
    assert _layers(a, False) == _layers(b, False)
    assert _layers(a, True) == _layers(b, True)
    for i in range(a.s.nchunks):
        ca, cb = a.chunk(i), b.chunk(i)
        assert isinstance(ca, np.ndarray) and np.array_equal(ca, cb), i
        if a.s.chunksize == 0:   # variable chunk sizes: the chunk's own nbytes
            n = int(ca[4:8].view(np.int32)[0])
        else:
            n = a.s.chunksize if i < a.s.nchunks - 1 or a.s.nbytes % a.s.chunksize == 0 else a.s.nbytes % a.s.chunksize
        ra, da = a.decompress_chunk(i, n)
        rb, db = b.decompress_chunk(i, n)
        assert ra == rb == n and np.array_equal(da, db), i
    if a.s.chunksize == 0:
        return   # slices need a fixed chunksize (schunk.c:1662-1700)
    ts = a.s.typesize
    nitems = a.s.nbytes // ts
    for start, stop in ((0, nitems), (nitems // 3, nitems // 3 + 5000), (nitems - 7, nitems)):
        start, stop = max(0, start), min(nitems, stop)
        ra, sa = a.get_slice(start, stop)
        rb, sb = b.get_slice(start, stop)
        assert ra == rb and np.array_equal(sa, sb), (start, stop)


def _from_buffer(L, buf, copy):
    p = L.blosc2_schunk_from_buffer(buf.ctypes.data, buf.nbytes, copy)
    assert p, "blosc2_schunk_from_buffer returned NULL"
    sc = B.SChunk.wrap(p, L)
    sc._keep = buf   # a frame-attached super-chunk reads the caller's buffer for its lifetime
    return sc


@pytest.mark.parametrize("copy", [False, True], ids=["attached", "copy"])
@pytest.mark.parametrize("name", FRAMES)
def test_from_buffer_matches_reference(name, copy):
    L, R = B.bind_schunk(B.lib()), _ref()
    buf = np.fromfile(os.path.join(GOLD, name + ".b2frame"), np.uint8)
    a, b = _from_buffer(L, buf, copy), _from_buffer(R, buf.copy(), copy)
    try:
        _same(a, b)
    finally:
        a.free()
        b.free()


@pytest.mark.parametrize("name", FRAMES)
def test_open_file_matches_reference(name, tmp_path):
    L, R = B.bind_schunk(B.lib()), _ref()
    path = os.path.join(GOLD, name + ".b2frame")
    a, b = L.blosc2_schunk_open(path.encode()), R.blosc2_schunk_open(path.encode())
    assert a and b
    a, b = B.SChunk.wrap(a, L), B.SChunk.wrap(b, R)
    try:
        _same(a, b)
    finally:
        a.free()
        b.free()
    # a frame embedded at an offset in a bigger file (blosc2_schunk_open_offset)
    blob = tmp_path / "embedded.bin"
    pad = b"\x00" * 4096
    blob.write_bytes(pad + open(path, "rb").read())
    a = L.blosc2_schunk_open_offset(str(blob).encode(), len(pad))
    b = R.blosc2_schunk_open_offset(str(blob).encode(), len(pad))
    assert a and b
    a, b = B.SChunk.wrap(a, L), B.SChunk.wrap(b, R)
    try:
        _same(a, b)
    finally:
        a.free()
        b.free()


@pytest.mark.parametrize("how", ["open", "from_buffer_attached"])
def test_frame_attached_handles_are_read_only(how):
    """Writes to a frame-attached handle would only change the in-memory copy (the reference
    writes them back to the frame): every write entry point refuses them, the counters
    and chunks stay, and a copy (from_buffer(copy=True)) stays writable."""
    L = B.bind_schunk(B.lib())
    path = os.path.join(GOLD, FRAMES[0] + ".b2frame")
    buf = np.fromfile(path, np.uint8)
    a = B.SChunk.wrap(L.blosc2_schunk_open(path.encode()), L) if how == "open" else _from_buffer(L, buf, False)
    try:
        before = (a.s.nchunks, a.s.nbytes, a.s.cbytes)
        c0 = a.chunk(0)
        n0 = a.s.chunksize
        raw = np.zeros(n0, np.uint8)
        assert a.append_buffer(raw) == -12                 # BLOSC2_ERROR_INVALID_PARAM
        assert a.append_chunk(c0) == -12
        assert a.insert_chunk(0, c0) == -12
        assert a.update_chunk(0, c0) == -12
        assert a.delete_chunk(0) == -12
        assert (a.s.nchunks, a.s.nbytes, a.s.cbytes) == before
    finally:
        a.free()
    c = _from_buffer(L, buf, True)
    try:
        assert c.append_chunk(c.chunk(0)) != -12
    finally:
        c.free()


def test_open_rejects_what_the_reference_rejects(tmp_path):
    L, R = B.bind_schunk(B.lib()), _ref()
    assert not L.blosc2_schunk_open(str(tmp_path / "absent.b2frame").encode())
    junk = np.frombuffer(b"not a frame at all" * 10, np.uint8).copy()
    assert not L.blosc2_schunk_from_buffer(junk.ctypes.data, junk.nbytes, True)
    assert not R.blosc2_schunk_from_buffer(junk.ctypes.data, junk.nbytes, True)


def test_metalayers_written_by_reference(tmp_path):
    """A frame with two metalayers and two vlmetalayers, written by the reference."""
    from b2ctypes import cparams as rcp, dparams as rdp
    from datagen import gen_f32
    R = _ref()
    L = B.bind_schunk(B.lib())
    cp, dp = rcp(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1)), rdp()
    st = B.Storage(True, None, C.cast(C.pointer(cp), C.c_void_p), C.cast(C.pointer(dp), C.c_void_p), None)
    sc = R.blosc2_schunk_new(C.byref(st))
    assert sc
    m1 = np.frombuffer(b"\x93\x01\x02\x03shape", np.uint8).copy()
    m2 = np.arange(300, dtype=np.uint8)
    assert R.blosc2_meta_add(sc, b"b2nd", m1.ctypes.data, m1.nbytes) >= 0
    assert R.blosc2_meta_add(sc, b"extra", m2.ctypes.data, m2.nbytes) >= 0
    data = gen_f32(5, 3 * 65536 + 1000)
    for i in range(0, data.size, 65536):
        part = np.ascontiguousarray(data[i:i + 65536])
        assert R.blosc2_schunk_append_buffer(sc, part.ctypes.data, part.nbytes) > 0
    v1 = np.frombuffer(b"user attributes " * 20, np.uint8).copy()
    v2 = np.zeros(0, np.uint8)
    assert R.blosc2_vlmeta_add(sc, b"attrs", v1.ctypes.data, v1.nbytes, None) >= 0
    assert R.blosc2_vlmeta_add(sc, b"empty", v2.ctypes.data, 0, None) >= 0
    out = C.POINTER(C.c_uint8)()
    nf = C.c_bool()
    n = R.blosc2_schunk_to_buffer(sc, C.byref(out), C.byref(nf))
    assert n > 0
    frame = np.ctypeslib.as_array(out, (n,)).copy()
    R.blosc2_schunk_free(sc)
    for copy in (False, True):
        a, b = _from_buffer(L, frame, copy), _from_buffer(R, frame.copy(), copy)
        try:
            assert [x[0] for x in _layers(a, False)] == [b"b2nd", b"extra"]
            assert [x[0] for x in _layers(a, True)] == [b"attrs", b"empty"]
            _same(a, b)
        finally:
            a.free()
            b.free()
    path = tmp_path / "meta.b2frame"
    frame.tofile(path)
    a, b = L.blosc2_schunk_open(str(path).encode()), R.blosc2_schunk_open(str(path).encode())
    a, b = B.SChunk.wrap(a, L), B.SChunk.wrap(b, R)
    try:
        _same(a, b)
        raw = np.concatenate([a.decompress_chunk(i, 65536 * 4 if i < 3 else 4000)[1] for i in range(4)])
        assert np.array_equal(raw, data.view(np.uint8))
    finally:
        a.free()
        b.free()
