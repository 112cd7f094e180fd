"""CPU-side checks of the drop-in boundary (no GPU compute here).

* the library loads and exports every symbol include/*.h declares;
* struct layouts match the reference's x86-64 ABI (src/lz4mt.h:102-147);
* the headers compile as C and C++;
* init/result functions behave like the reference (src/lz4mt.cpp:851-895,
  src/lz4mt_result.cpp);
* the host frame engine (lz4mtCompress / lz4mtDecompress) driven by a
  plug-in CPU codec (liblz4 1.9.3 via the reference's own operator API)
  writes the golden frames and reports the reference's error codes;
* device entry points fail loudly without a GPU.
"""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, read_golden, with_stream_size

import lz4mt_amd as L
from lz4mt_amd import _abi

HEADERS = [os.path.join(ROOT, "include", h) for h in ("lz4mt.h", "lz4mt_hip.h", "lz4mt_io.h")]
LIBLZ4 = "/lib/x86_64-linux-gnu/liblz4.so.1"


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(lz4mt\w+)\s*\(", text, flags=re.M):
            if not m.group(0).lstrip().startswith("typedef"):
                names.add(m.group(1))
    return names


def test_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    declared = declared_functions()
    assert len(declared) >= 30
    missing = declared - exported
    assert not missing, missing
    assert declared == set(_abi.PROTOTYPES), declared ^ set(_abi.PROTOTYPES)


def test_struct_layout_matches_reference_abi():
    C = _abi.Lz4MtContext
    assert ctypes.sizeof(C) == 96
    offs = {n: getattr(C, n).offset for n, _ in C._fields_}
    assert offs == {"result": 0, "readCtx": 8, "read": 16, "readSkippable": 24, "readSeek": 32, "readEof": 40,
                    "writeCtx": 48, "write": 56, "compress": 64, "compressBound": 72, "decompress": 80,
                    "mode": 88, "compressionLevel": 92}
    S = _abi.Lz4MtStreamDescriptor
    assert ctypes.sizeof(S) == 32
    assert (S.flg.offset, S.bd.offset, S.streamSize.offset, S.dictId.offset) == (0, 7, 16, 24)


@pytest.mark.parametrize("compiler,ext", [("gcc", "c"), ("g++", "cpp")])
def test_headers_compile(tmp_path, compiler, ext):
    src = tmp_path / f"t.{ext}"
    src.write_text('#include "lz4mt.h"\n#include "lz4mt_hip.h"\n#include "lz4mt_io.h"\n'
                   "_Static_assert(sizeof(Lz4MtContext) == 96, \"ctx\");\n" if ext == "c" else
                   '#include "lz4mt.h"\n#include "lz4mt_hip.h"\n#include "lz4mt_io.h"\n'
                   "static_assert(sizeof(Lz4MtContext) == 96, \"ctx\");\n"
                   "static_assert(sizeof(Lz4MtStreamDescriptor) == 32, \"sd\");\n")
    subprocess.run([compiler, "-Wall", "-Werror", "-c", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(tmp_path / "t.o")], check=True)


def test_init_functions():
    c = L.init_context()
    assert c.result == 0 and c.mode == L.MODE_PARALLEL and c.compressionLevel == 0
    assert not any([c.read, c.write, c.compress, c.decompress, c.readEof, c.readSeek, c.readSkippable])
    sd = L.init_stream_descriptor()
    assert (sd.flg.streamChecksum, sd.flg.blockIndependence, sd.flg.versionNumber, sd.bd.blockMaximumSize) == \
        (1, 1, 1, 7)
    assert (sd.flg.blockChecksum, sd.flg.streamSize, sd.flg.presetDictionary, sd.streamSize, sd.dictId) == \
        (0, 0, 0, 0, 0)


def test_result_strings_and_exit_codes():
    # the reference's table (src/lz4mt_result.cpp:4-89) has no case for 16,
    # 24 and 25: they print "Unknown code" there
    unnamed = {16, 24, 25}
    for i, name in enumerate(L.RESULT_NAMES):
        assert L.result_to_string(i) == ("Unknown code" if i in unnamed else name), i
    assert L.result_to_string(99) == "Unknown code"
    assert L.result_to_string(-1) == "Unknown code"
    expect = {0: 0, 1: 1, 2: 44, 3: 61, 4: 66, 5: 1, 6: 62, 7: 69, 8: 68, 9: 32, 10: 37, 11: 37, 12: 71, 13: 73,
              14: 74, 15: 74, 16: 75, 17: 75, 18: 77, 19: 1, 20: 72, 21: 65, 22: 67, 23: 67, 24: 42, 25: 43,
              26: 76, 27: 78}
    for code, e in expect.items():
        assert L.result_to_exit_code(code) == e, code


def test_device_entry_points_fail_without_gpu():
    if L.device_count() > 0:
        pytest.skip("a HIP device is present")
    assert L.lib.lz4mtHipCompressBlock(b"abcdabcdabcdabcd", ctypes.create_string_buffer(64), 16, 16, 0) < 0
    sd = L.init_stream_descriptor()
    r = L.lib.lz4mtHipCompressFrame(None, 0, ctypes.c_void_p(1), 1 << 20, None, ctypes.byref(sd), None, 0, None)
    assert r == L.Result.ERROR


# ---------------------------------------------------------------------------
# host frame engine with a plug-in CPU codec (the reference's operator API)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def cpu_codec():
    if not os.path.exists(LIBLZ4):
        pytest.skip("liblz4 not present")
    lz = ctypes.CDLL(LIBLZ4)

    def comp(src, dst, n, cap, level):
        return lz.LZ4_compress_limitedOutput(ctypes.c_void_p(src), ctypes.c_void_p(dst), n, cap)

    def decomp(src, dst, n, cap):
        return lz.LZ4_decompress_safe(ctypes.c_void_p(src), ctypes.c_void_p(dst), n, cap)
    return comp, decomp


@pytest.mark.parametrize("mode", [L.MODE_SEQUENTIAL, L.MODE_PARALLEL])
def test_host_engine_writes_golden_frames(golden, golden_inputs, cpu_codec, mode):
    comp, decomp = cpu_codec
    for f in golden["frames"]:
        if golden_inputs[f["input"]].__len__() > 70_000 and f["bid"] == 4:
            continue   # keep the CPU suite fast
        data = golden_inputs[f["input"]]
        sd = L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"])
        r, frame = L.compress(data, sd, mode=mode, compress_cb=comp)
        assert r == 0, (f["file"], L.result_to_string(r))
        assert frame == read_golden(f["file"]), f["file"]
        r, out, sd2 = L.decompress(frame, len(data) + 64, mode=mode, decompress_cb=decomp)
        assert r == 0 and out == data, (f["file"], L.result_to_string(r))
        assert (sd2.bd.blockMaximumSize, sd2.flg.blockChecksum, sd2.flg.streamChecksum) == \
            (f["bid"], int(f["block_checksum"]), int(f["stream_checksum"]))


def test_host_engine_error_codes(golden_inputs, cpu_codec):
    comp, decomp = cpu_codec
    data = golden_inputs["syn300k"]
    r, f = L.compress(data, L.make_sd(5, True, True), compress_cb=comp)
    assert r == 0

    def dec(b):
        return L.decompress(b, len(data) + 64, mode=L.MODE_SEQUENTIAL, decompress_cb=decomp)[0]
    R = L.Result
    assert dec(f) == R.OK
    assert dec(b"\x01\x02\x03\x04rest") == R.INVALID_MAGIC_NUMBER
    bad = bytearray(f); bad[6] ^= 1
    assert dec(bytes(bad)) == R.INVALID_HEADER_CHECKSUM
    bad = bytearray(f); bad[4] &= 0x3F
    assert dec(bytes(bad)) == R.INVALID_VERSION
    bad = bytearray(f); bad[5] = 0x30
    assert dec(bytes(bad)) == R.INVALID_BLOCK_MAXIMUM_SIZE
    bad = bytearray(f); bad[20] ^= 0xFF
    assert dec(bytes(bad)) in (R.BLOCK_CHECKSUM_MISMATCH, R.DECOMPRESS_FAIL)
    assert dec(f[:-2]) == R.CANNOT_READ_STREAM_CHECKSUM
    assert dec(f[:100]) == R.CANNOT_READ_BLOCK_DATA
    bad = bytearray(f); bad[-1] ^= 1
    assert dec(bytes(bad)) == R.STREAM_CHECKSUM_MISMATCH
    skip = (0x184D2A51).to_bytes(4, "little") + (5).to_bytes(4, "little") + b"12345"
    r, out, _ = L.decompress(f + skip + f + b"junkjunk", 2 * len(data) + 64, decompress_cb=decomp)
    assert r == R.OK and out == data + data
    # block-dependent frames run on the device engine only (the reference
    # bypasses ctx.compress for them): without a GPU they fail loudly
    if L.device_count() == 0:
        sd = L.make_sd(7, block_dependence=True)
        assert L.compress(b"abc", sd, compress_cb=comp)[0] == R.ERROR


def test_cstdio_adapters(tmp_path, golden_inputs, cpu_codec):
    comp, decomp = cpu_codec
    data = golden_inputs["text20k"]
    src, dst = tmp_path / "in.bin", tmp_path / "out.lz4"
    src.write_bytes(data)
    ctx = L.init_context()
    keep = [_abi.COMPRESS_FN(comp)]
    ctx.compress = ctypes.cast(keep[0], ctypes.c_void_p)
    L.lib.lz4mtIoBindCstdio(ctypes.byref(ctx))
    assert L.lib.lz4mtIoOpenIstream(ctypes.byref(ctx), str(src).encode())
    assert L.lib.lz4mtIoOpenOstream(ctypes.byref(ctx), str(dst).encode(), 0)
    sd = L.init_stream_descriptor()
    assert L.lib.lz4mtCompress(ctypes.byref(ctx), ctypes.byref(sd)) == 0
    L.lib.lz4mtIoCloseIstream(ctypes.byref(ctx))
    L.lib.lz4mtIoCloseOstream(ctypes.byref(ctx))
    assert dst.read_bytes() == read_golden("frames/text20k.B7Sx.lz4")
    assert L.lib.lz4mtIoGetFilesize(str(dst).encode()) == dst.stat().st_size


def test_large_transfers_through_io_bindings(tmp_path):
    """Large reads/writes go through the copy pool (parallel memcpy /
    pread / pwrite); bytes, positions and fread/feof semantics must not change."""
    import random
    rnd = random.Random(7)
    data = bytes(rnd.getrandbits(8) for _ in range(1 << 16)) * 150 + b"tail!"   # 9.4 MiB
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    src.write_bytes(data)
    ctx = L.init_context()
    L.lib.lz4mtIoBindCstdio(ctypes.byref(ctx))
    assert L.lib.lz4mtIoOpenIstream(ctypes.byref(ctx), str(src).encode())
    assert L.lib.lz4mtIoOpenOstream(ctypes.byref(ctx), str(dst).encode(), 0)
    got = []
    for size in (5, 3 << 20, 4096, 4 << 20, 4 << 20):   # small, large, small, large, short-at-EOF
        buf = ctypes.create_string_buffer(size)
        n = L.lib.lz4mtIoRead(ctypes.byref(ctx), buf, size)
        got.append(buf.raw[:n])
        assert L.lib.lz4mtIoWrite(ctypes.byref(ctx), buf, n) == n
    assert b"".join(got) == data
    assert L.lib.lz4mtIoReadEof(ctypes.byref(ctx)) != 0
    buf = ctypes.create_string_buffer(8)
    assert L.lib.lz4mtIoRead(ctypes.byref(ctx), buf, 8) == 0
    L.lib.lz4mtIoCloseIstream(ctypes.byref(ctx))
    L.lib.lz4mtIoCloseOstream(ctypes.byref(ctx))
    assert dst.read_bytes() == data

    # memory binding: the same sequence of reads and writes
    inb = ctypes.create_string_buffer(data, len(data))
    outb = ctypes.create_string_buffer(len(data) + 16)
    io = _abi.Lz4MtMemIo(ctypes.cast(inb, ctypes.c_void_p).value, len(data), 0, 0,
                         ctypes.cast(outb, ctypes.c_void_p).value, len(data) + 16, 0)
    ctx = L.init_context()
    L.lib.lz4mtMemBind(ctypes.byref(ctx), ctypes.byref(io))
    rd, wr = _abi.READ_FN(ctx.read), _abi.WRITE_FN(ctx.write)
    for size in (5, 3 << 20, 4096, 4 << 20, 4 << 20):
        buf = ctypes.create_string_buffer(size)
        n = rd(ctypes.byref(ctx), ctypes.cast(buf, ctypes.c_void_p), size)
        assert wr(ctypes.byref(ctx), ctypes.cast(buf, ctypes.c_void_p), n) == n
    assert io.eof == 1 and io.inPos == len(data) and io.outPos == len(data)
    assert outb.raw[:len(data)] == data


def test_copy_pool_split_keeps_the_last_bytes(tmp_path):
    """Transfers whose size over the piece count is a whole number of pages
    plus a remainder (with 8 pieces: 1 MiB + 1, 2 MiB + 1, 3 MiB + 2, ...):
    every byte lands, by the memory and the cstdio bindings."""
    import random
    sizes = [(1 << 20) + 1, (2 << 20) + 1, (3 << 20) + 2, (4 << 20) + 3, (8 << 20) + 7, (2 << 20) + 4097]
    rnd = random.Random(11)
    data = rnd.randbytes(sum(sizes))
    inb = ctypes.create_string_buffer(data, len(data))
    outb = ctypes.create_string_buffer(len(data))
    io = _abi.Lz4MtMemIo(ctypes.cast(inb, ctypes.c_void_p).value, len(data), 0, 0,
                         ctypes.cast(outb, ctypes.c_void_p).value, len(data), 0)
    ctx = L.init_context()
    L.lib.lz4mtMemBind(ctypes.byref(ctx), ctypes.byref(io))
    rd, wr = _abi.READ_FN(ctx.read), _abi.WRITE_FN(ctx.write)
    pos = 0
    for size in sizes:
        buf = ctypes.create_string_buffer(size)
        assert rd(ctypes.byref(ctx), ctypes.cast(buf, ctypes.c_void_p), size) == size
        assert buf.raw == data[pos:pos + size], size
        assert wr(ctypes.byref(ctx), ctypes.cast(buf, ctypes.c_void_p), size) == size
        pos += size
    assert outb.raw == data

    src = tmp_path / "in.bin"
    src.write_bytes(data)
    ctx = L.init_context()
    L.lib.lz4mtIoBindCstdio(ctypes.byref(ctx))
    assert L.lib.lz4mtIoOpenIstream(ctypes.byref(ctx), str(src).encode())
    pos = 0
    for size in sizes:
        buf = ctypes.create_string_buffer(size)
        assert L.lib.lz4mtIoRead(ctypes.byref(ctx), buf, size) == size
        assert buf.raw == data[pos:pos + size], size
        pos += size
    L.lib.lz4mtIoCloseIstream(ctypes.byref(ctx))


@pytest.mark.parametrize("mode", [L.MODE_SEQUENTIAL, L.MODE_PARALLEL])
def test_host_engine_stream_size_field(golden_inputs, cpu_codec, mode):
    """FLG.3 (content size): header written as the reference does, frame
    decodes and reports the size back in the descriptor."""
    comp, decomp = cpu_codec
    data = golden_inputs["text20k"]
    plain = L.compress(data, L.make_sd(7, True, True), mode=mode, compress_cb=comp)[1]
    sd = L.make_sd(7, True, True)
    sd.flg.streamSize = 1
    sd.streamSize = len(data)
    r, frame = L.compress(data, sd, mode=mode, compress_cb=comp)
    assert r == 0 and frame == with_stream_size(plain, len(data))
    r, out, sd2 = L.decompress(frame, len(data) + 64, mode=mode, decompress_cb=decomp)
    assert r == 0 and out == data and sd2.flg.streamSize == 1 and sd2.streamSize == len(data)


def test_large_writes_to_append_mode_file(tmp_path):
    """An O_APPEND output (a caller's own FILE*) keeps fwrite order: large
    writes are not split into positional pieces there."""
    import random
    rnd = random.Random(3)
    base = bytes(rnd.getrandbits(8) for _ in range(1 << 12))
    chunks = [bytes([i]) + base * (3072 + i) for i in range(6)]   # 12+ MiB each: split into 8 pieces if positional
    dst = tmp_path / "out.bin"
    dst.write_bytes(b"head")
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    fp = libc.fopen(str(dst).encode(), b"ab")
    assert fp
    ctx = L.init_context()
    L.lib.lz4mtIoBindCstdio(ctypes.byref(ctx))
    ctx.writeCtx = fp
    for c in chunks:
        assert L.lib.lz4mtIoWrite(ctypes.byref(ctx), c, len(c)) == len(c)
    libc.fclose(fp)
    assert dst.read_bytes() == b"head" + b"".join(chunks)


def _ref_bd_plan(bid, sizes, ref_buffer):
    """compressBlockDependency's buffer loop (reference src/lz4mt.cpp:460-538:
    max(bm + 64 KiB, 1088 KiB) input buffer, translate() when the next block
    would not fit) over lz4 1.9.3's LZ4_compress_fast_continue dictionary
    bookkeeping, restated on buffer offsets, with the buffer's CONTENT
    tracked byte range by byte range: for each block, what the encoder
    needs in block coordinates (block at 65536) -- catch-up bounds for
    candidates in the block / the history, the dictSmall limit -- and
    whether the history bytes lz4 reads are the stream's own previous bytes
    (shift 0), the block's own bytes (shift = where they start + 65536), or
    neither (None).  ref_buffer = False: 1 and 4 MiB blocks in one
    contiguous buffer (the decodable stream); 64 / 256 KiB always buffered."""
    bm = 1 << (8 + 2 * bid)
    buffered = bid <= 5 or ref_buffer
    size = max(bm + 65536, 1088 * 1024) if buffered else 1 << 62
    seg = []                      # (buf_lo, buf_hi, stream_lo): what the buffer holds
    dic, dsz, cur = None, 0, 0    # LZ4_stream_t: dictionary (buffer offset or NULL), dictSize, currentOffset
    ins, pos, out = 0, 0, []

    def stored(x):
        for lo, hi, s in reversed(seg):
            if lo <= x < hi:
                return s + (x - lo)
        return None

    for n in sizes:
        if ins + bm > size:   # translate(): LZ4_slideInputBuffer returns the dictionary pointer (1.9.3)
            ins = dic
        seg.append((ins, ins + n, pos))
        dend = (dic or 0) + dsz
        if cur + n > 0x80000000:   # LZ4_renormDictT
            cur = 65536
            dsz = min(dsz, 65536)
            dic = dend - dsz
        if 0 < dsz < 4 and (dic is None or dend != ins):   # tiny dictionaries
            dsz, dic, dend = 0, ins, ins
        if dic is not None and ins + n > dic and ins + n < dend:   # input overlaps the dictionary
            dsz = dend - (ins + n)
            dsz = 0 if dsz < 4 else min(dsz, 65536)
            dic = dend - dsz
        prefix = dic is not None and dend == ins
        small = dsz < 65536 and dsz < cur
        ds = min(dsz, 65536)
        # the buffer -> stream map is linear between segment edges: checking
        # the history range at every edge inside it (and its ends) checks it all
        lo_h, hi_h = dend - ds, dend
        xs = {lo_h, hi_h - 1} | {e + d for a, b, _ in seg for e in (a, b) for d in (-1, 0)
                                 if lo_h <= e + d < hi_h}
        if ds == 0 or all(stored(x) == pos - (dend - x) for x in xs):
            shift = 0
        elif ins <= lo_h and hi_h <= ins + n:
            shift = dend - ins
        else:
            shift = None
        out.append((65536 - ds if prefix else 65536, 65536 - ds, 65536 - ds if small else 0, shift))
        cur += n
        if prefix:
            dsz += n
        else:
            dic, dsz = ins, n
        ins += n
        pos += n
    return out


@pytest.mark.parametrize("bid", [4, 5, 6, 7])
@pytest.mark.parametrize("ref_buffer", [False, True])
def test_bd_plan_matches_the_reference_buffer_loop(bid, ref_buffer):
    """BdSim (lz4mt_host.h, the host half of the -BD encode, exported as
    lz4mtDebugBdPlan) against the restatement above on full, short and
    ragged block sequences: lz4's modes and bounds per block, and where the
    history the encoder must read stands.  With the reference's buffer at 1
    and 4 MiB (ref_buffer) every full block after the first reads its own
    bytes (shift = the block size); 64 / 256 KiB blocks and the contiguous
    stream always read the true history."""
    import random
    import ctypes
    bm = 1 << (8 + 2 * bid)
    rnd = random.Random(bid * 2 + ref_buffer)
    cases = [[bm] * 9, [bm] * 4 + [bm // 3], [bm, 100, bm, bm, 7, bm], [bm // 2] * 5 + [bm] * 3,
             [rnd.choice([bm, bm, bm, rnd.randrange(1, bm)]) for _ in range(40)], [3, bm, 2, bm, bm]]
    for sizes in cases:
        want = _ref_bd_plan(bid, sizes, ref_buffer)
        arr = (ctypes.c_uint32 * len(sizes))(*sizes)
        plan = (ctypes.c_uint32 * (4 * len(sizes)))()
        rc = L.lib.lz4mtDebugBdPlan(bid, 1 if ref_buffer else 0, arr, len(sizes), plan)
        got = [tuple(plan[4 * i:4 * i + 4]) for i in range(len(sizes))]
        bad = any(w[3] is None for w in want)
        assert rc == (1 if bad else 0), (sizes[:8], rc)
        for i, (w, g) in enumerate(zip(want, got)):
            assert g[:3] == w[:3], (bid, ref_buffer, i, sizes[:8], g, w)
            if w[3] is not None:
                assert g[3] == (w[3] if ref_buffer else 0), (bid, ref_buffer, i, g, w)
        if ref_buffer and bid >= 6 and sizes == [bm] * 9:
            assert [g[3] for g in got] == [0] + [bm] * 8
        if not ref_buffer or bid <= 5:
            assert all(w[3] == 0 for w in want), (bid, sizes[:8])


def _device_functions(lib_path, tmp_path):
    """Names of the outlined (called, not inlined) gfx950 functions in every
    code object bundle of the library's .hip_fatbin section."""
    bundler = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not (os.path.exists(bundler) and os.path.exists(readelf)):
        pytest.skip("ROCm LLVM tools absent")
    fat = tmp_path / "fat.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib_path, str(fat)], check=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__|CCOB", data)] + [len(data)]
    names = []
    for i, (a, b) in enumerate(zip(offs, offs[1:])):
        part, co = tmp_path / f"b{i}.bin", tmp_path / f"co{i}.o"
        part.write_bytes(data[a:b])
        subprocess.run([bundler, "--type=o", f"--input={part}", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        out = subprocess.run([readelf, "-s", "--wide", str(co)], check=True, capture_output=True, text=True).stdout
        names += [ln.split()[-1] for ln in out.splitlines() if " FUNC " in ln]
    assert names, "no gfx950 code object found"
    return names


def test_frame_encoders_are_inlined(tmp_path):
    """The frame path's block encoders (k_encode, k_encode_p17, k_encode16,
    k_encode_pub) run encode_block_v5 inlined: a second call site of one of
    their instantiations (a debug kernel, say) makes LLVM outline it into a
    called function, which cost k_encode ~8 % when it happened in round 4.
    Only the -BD (LINK) instantiations are meant to be called functions."""
    funcs = _device_functions(os.path.join(ROOT, "lz4mt_amd", "liblz4mt_amd.so"), tmp_path)
    outlined = [f for f in funcs if "encode_block_v5" in f]
    # template arguments <ST, U16, SPLIT, LINK, ...> mangle as ILb<ST>ELb<U16>ELb<SPLIT>ELb<LINK>E
    bad = [f for f in outlined if not re.search(r"encode_block_v5ILb\dELb\dELb\dELb1E", f)]
    assert not bad, f"frame encoders outlined: {bad}"
