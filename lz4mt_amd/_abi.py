"""ctypes view of the liblz4mt_amd.so C ABI (include/lz4mt.h, lz4mt_hip.h, lz4mt_io.h).

Struct layouts mirror the reference header (src/lz4mt.h:102-147); the ABI
test (tests/test_abi.py) checks every offset against the x86-64 layout the
reference compiles to: Lz4MtContext 96 B, Lz4MtStreamDescriptor 32 B.
"""
import ctypes
import os

c_int, c_uint32, c_uint64, c_size_t, c_void_p, c_char_p, c_float = (
    ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p,
    ctypes.c_float)

LIB_NAME = "liblz4mt_amd.so"
LIB_PATH = os.environ.get("LZ4MT_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

# Lz4MtMode (src/lz4mt.h:61-66) + the DEVICE extension bit
MODE_PARALLEL = 0
MODE_SEQUENTIAL = 1
MODE_DEVICE = 2

RESULT_NAMES = [
    "OK", "ERROR", "INVALID_MAGIC_NUMBER", "INVALID_HEADER", "PRESET_DICTIONARY_IS_NOT_SUPPORTED_YET",
    "BLOCK_DEPENDENCE_IS_NOT_SUPPORTED_YET", "INVALID_VERSION", "INVALID_HEADER_CHECKSUM",
    "INVALID_BLOCK_MAXIMUM_SIZE", "CANNOT_WRITE_HEADER", "CANNOT_WRITE_EOS", "CANNOT_WRITE_STREAM_CHECKSUM",
    "CANNOT_READ_BLOCK_SIZE", "CANNOT_READ_BLOCK_DATA", "CANNOT_READ_BLOCK_CHECKSUM",
    "CANNOT_READ_STREAM_CHECKSUM", "BLOCK_CHECKSUM_MISMATCH", "STREAM_CHECKSUM_MISMATCH", "DECOMPRESS_FAIL",
    "BAD_ARG", "INVALID_BLOCK_SIZE", "INVALID_HEADER_RESERVED1", "INVALID_HEADER_RESERVED2",
    "INVALID_HEADER_RESERVED3", "INVALID_HEADER_SKIPPABLE_SIZE_UNREADABLE",
    "INVALID_HEADER_CANNOT_SKIP_SKIPPABLE_AREA", "CANNOT_WRITE_DATA_BLOCK", "CANNOT_WRITE_DECODED_BLOCK",
]
Result = type("Result", (), {name: i for i, name in enumerate(RESULT_NAMES)})


class Lz4MtFlg(ctypes.Structure):
    _fields_ = [("presetDictionary", ctypes.c_byte), ("reserved1", ctypes.c_byte),
                ("streamChecksum", ctypes.c_byte), ("streamSize", ctypes.c_byte),
                ("blockChecksum", ctypes.c_byte), ("blockIndependence", ctypes.c_byte),
                ("versionNumber", ctypes.c_byte)]


class Lz4MtBd(ctypes.Structure):
    _fields_ = [("reserved3", ctypes.c_byte), ("blockMaximumSize", ctypes.c_byte), ("reserved2", ctypes.c_byte)]


class Lz4MtStreamDescriptor(ctypes.Structure):
    _fields_ = [("flg", Lz4MtFlg), ("bd", Lz4MtBd), ("streamSize", c_uint64), ("dictId", c_uint32)]


class Lz4MtContext(ctypes.Structure):
    pass


READ_FN = ctypes.CFUNCTYPE(c_int, ctypes.POINTER(Lz4MtContext), c_void_p, c_int)
READ_SKIPPABLE_FN = ctypes.CFUNCTYPE(c_int, ctypes.POINTER(Lz4MtContext), c_uint32, c_size_t)
READ_SEEK_FN = ctypes.CFUNCTYPE(c_int, ctypes.POINTER(Lz4MtContext), c_int)
READ_EOF_FN = ctypes.CFUNCTYPE(c_int, ctypes.POINTER(Lz4MtContext))
WRITE_FN = ctypes.CFUNCTYPE(c_int, ctypes.POINTER(Lz4MtContext), c_void_p, c_int)
COMPRESS_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_int, c_int, c_int)
COMPRESS_BOUND_FN = ctypes.CFUNCTYPE(c_int, c_int)
DECOMPRESS_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_int, c_int)

Lz4MtContext._fields_ = [
    ("result", c_int), ("readCtx", c_void_p), ("read", c_void_p), ("readSkippable", c_void_p),
    ("readSeek", c_void_p), ("readEof", c_void_p), ("writeCtx", c_void_p), ("write", c_void_p),
    ("compress", c_void_p), ("compressBound", c_void_p), ("decompress", c_void_p), ("mode", c_int),
    ("compressionLevel", c_int),
]


class Lz4MtMemIo(ctypes.Structure):
    _fields_ = [("in_", c_void_p), ("inSize", c_uint64), ("inPos", c_uint64), ("eof", c_int),
                ("out", c_void_p), ("outCap", c_uint64), ("outPos", c_uint64)]


CTX_P = ctypes.POINTER(Lz4MtContext)
SD_P = ctypes.POINTER(Lz4MtStreamDescriptor)

# name -> (restype, argtypes); every symbol include/*.h declares
PROTOTYPES = {
    # lz4mt.h (reference src/lz4mt.h:150-163)
    "lz4mtInitContext": (Lz4MtContext, []),
    "lz4mtInitStreamDescriptor": (Lz4MtStreamDescriptor, []),
    "lz4mtResultToString": (c_char_p, [c_int]),
    "lz4mtResultToLz4cExitCode": (c_int, [c_int]),
    "lz4mtCompress": (c_int, [CTX_P, SD_P]),
    "lz4mtDecompress": (c_int, [CTX_P, SD_P]),
    # lz4mt_hip.h
    "lz4mtHipCompressBlock": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int]),
    "lz4mtHipCompressBound": (c_int, [c_int]),
    "lz4mtHipDecompressBlock": (c_int, [c_void_p, c_void_p, c_int, c_int]),
    "lz4mtHipFrameBound": (c_uint64, [c_uint64, SD_P]),
    "lz4mtHipCompressWorkspaceSize": (c_uint64, [c_uint64, SD_P]),
    "lz4mtHipCompressFrame": (c_int, [c_void_p, c_uint64, c_void_p, c_uint64, ctypes.POINTER(c_uint64), SD_P,
                                      c_void_p, c_uint64, c_void_p]),
    "lz4mtHipCompressFrameAsync": (c_int, [c_void_p, c_uint64, c_void_p, c_uint64, c_void_p, SD_P, c_void_p,
                                           c_uint64, c_void_p]),
    "lz4mtHipCompressWorkspaceSizeEx": (c_uint64, [c_uint64, SD_P, c_int]),
    "lz4mtHipCompressFrameEx": (c_int, [c_void_p, c_uint64, c_void_p, c_uint64, ctypes.POINTER(c_uint64), SD_P,
                                        c_int, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipCompressFrameAsyncEx": (c_int, [c_void_p, c_uint64, c_void_p, c_uint64, c_void_p, SD_P, c_int,
                                             c_void_p, c_uint64, c_void_p]),
    "lz4mtHipFrameInfo": (c_int, [c_void_p, c_uint64, SD_P, ctypes.POINTER(c_uint64), ctypes.POINTER(c_uint64),
                                  c_void_p]),
    "lz4mtHipDecompressFrame": (c_int, [c_void_p, c_uint64, c_void_p, c_uint64, ctypes.POINTER(c_uint64), SD_P,
                                        c_void_p]),
    "lz4mtHipStreamBound": (c_int, [c_void_p, c_uint64, ctypes.POINTER(c_uint64), c_void_p]),
    "lz4mtHipFrameRecords": (c_int, [c_void_p, c_uint64, ctypes.POINTER(c_uint64), c_uint64,
                                     ctypes.POINTER(c_uint64), ctypes.POINTER(c_int), SD_P, c_void_p]),
    "lz4mtHipGenSynthetic": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p]),
    "lz4mtHipXxh32Chunks": (c_int, [c_void_p, c_uint64, c_uint32, c_void_p, c_void_p]),
    "lz4mtHipXxh32": (c_uint32, [c_void_p, c_uint64, c_void_p]),
    "lz4mtHipDeviceCount": (c_int, []),
    "lz4mtHipReleaseCaches": (None, []),
    "lz4mtHipSetTiming": (None, [c_int]),
    "lz4mtHipGetTimings": (c_int, [ctypes.POINTER(c_float)]),
    "lz4mtHipShardWorkspaceSize": (c_uint64, [c_uint64, SD_P]),
    "lz4mtHipShardPackBound": (c_uint64, [c_uint64, SD_P, c_uint32]),
    "lz4mtHipFrameHeader": (c_int, [SD_P, c_void_p]),
    "lz4mtHipShardReset": (c_int, [c_uint64, SD_P, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipShardEncode": (c_int, [c_void_p, c_uint64, SD_P, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipShardRelease": (None, [c_void_p]),
    "lz4mtHipShardPack": (c_int, [c_void_p, c_uint64, SD_P, c_void_p, c_uint64, c_void_p, c_uint64, c_uint32, c_int,
                                  c_void_p]),
    "lz4mtHipShardUnpack": (c_int, [c_void_p, c_uint64, SD_P, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipShardAssemble": (c_int, [c_void_p, c_uint64, SD_P, c_void_p, c_uint64, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipIpcAlloc": (c_int, [c_uint64, ctypes.POINTER(c_void_p), c_void_p]),
    "lz4mtHipIpcAllocKind": (c_int, [c_uint64, ctypes.POINTER(c_void_p), c_void_p, c_int, ctypes.POINTER(c_int)]),
    "lz4mtHipDevicePciBusId": (c_int, [c_int, c_char_p, c_int]),
    "lz4mtHipDeviceByPciBusId": (c_int, [c_char_p]),
    "lz4mtHipCanAccessPeer": (c_int, [c_int, c_int]),
    "lz4mtHipIpcOpen": (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    "lz4mtHipIpcClose": (c_int, [c_void_p]),
    "lz4mtHipFree": (c_int, [c_void_p]),
    "lz4mtHipCopyAsync": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipShardBodyBytes": (c_uint64, [c_uint64, SD_P, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipDebugEncodeStats": (c_int, [c_void_p, c_uint64, c_uint32, ctypes.POINTER(c_uint64), c_void_p]),
    "lz4mtHipDebugEncodeBlockStats": (c_int, [c_void_p, c_uint64, c_uint32, ctypes.POINTER(c_uint64), c_void_p]),
    "lz4mtHipDebugEncode": (c_int, [c_void_p, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p]),
    "lz4mtHipCheckEncoderOrder": (c_int, []),
    "lz4mtHipEncoderProbe": (c_int, []),
    "lz4mtHipDebugEncodeOverlap": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_void_p, c_void_p]),
    "lz4mtDebugBdPlan": (c_int, [c_int, c_int, c_void_p, c_uint64, c_void_p]),
    "lz4mtHipDebugFetchCal": (c_int, [c_void_p, c_uint64, c_int, c_void_p, c_void_p]),
    "lz4mtHipDebugDecodeStats": (c_int, [c_void_p, c_uint64, ctypes.POINTER(c_uint64), c_void_p]),
    # lz4mt_io.h
    "lz4mtIoOpenIstream": (c_int, [CTX_P, c_char_p]),
    "lz4mtIoOpenOstream": (c_int, [CTX_P, c_char_p, c_int]),
    "lz4mtIoCloseIstream": (None, [CTX_P]),
    "lz4mtIoCloseOstream": (None, [CTX_P]),
    "lz4mtIoBindCstdio": (None, [CTX_P]),
    "lz4mtIoRead": (c_int, [CTX_P, c_void_p, c_int]),
    "lz4mtIoReadSkippable": (c_int, [CTX_P, c_uint32, c_size_t]),
    "lz4mtIoReadSeek": (c_int, [CTX_P, c_int]),
    "lz4mtIoReadEof": (c_int, [CTX_P]),
    "lz4mtIoWrite": (c_int, [CTX_P, c_void_p, c_int]),
    "lz4mtIoGetFilesize": (c_uint64, [c_char_p]),
    "lz4mtMemBind": (None, [CTX_P, ctypes.POINTER(Lz4MtMemIo)]),
}


def load(path=LIB_PATH):
    """Loads the library and attaches prototypes.  Raises if it is missing."""
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built: run `make` (or __graft_entry__.build()) first")
    lib = ctypes.CDLL(path)
    # an A/B build of an older tree (LZ4MT_AMD_LIB, tools/ab.sh) may predate
    # some entry points: those are skipped there, never for the product
    older_ok = os.environ.get("LZ4MT_AMD_LIB_OLDER") == "1" and path != os.path.join(
        os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
    for name, (res, args) in PROTOTYPES.items():
        if older_ok and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
