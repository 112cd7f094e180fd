"""Which receive-buffer memory kinds allocate AND export an IPC handle, by size
(the IPC push takes uncached memory only).  For each size:
hipExtMallocWithFlags(hipDeviceMallocUncached) and (hipDeviceMallocFinegrained)
and hipMalloc, then hipIpcGetMemHandle on each; prints the HIP error codes."""
import ctypes
import sys

import torch  # noqa: F401  (loads the HIP runtime)

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipFree.argtypes = [ctypes.c_void_p]
FINE, UNCACHED = 0x1, 0x3   # hipDeviceMallocFinegrained, hipDeviceMallocUncached
sizes = [int(x) for x in sys.argv[1:]] or [
    65536, 524288, 1 << 20, (1 << 20) + 4096, 1508160, 1573696, 2 << 20, (2 << 20) + 4096, 3 << 20, 4 << 20,
    (8 << 20) + 123, 64 << 20, 300 << 20]
for n in sizes:
    row = [f"{n:>10}"]
    for name, fl in (("uncached", UNCACHED), ("fine", FINE), ("plain", None)):
        p = ctypes.c_void_p()
        e = hip.hipMalloc(ctypes.byref(p), n) if fl is None else hip.hipExtMallocWithFlags(ctypes.byref(p), n, fl)
        h = (ctypes.c_uint8 * 64)()
        x = hip.hipIpcGetMemHandle(h, p) if e == 0 else -1
        if e == 0:
            hip.hipFree(p)
        row.append(f"{name}: alloc {e} ipc {x}")
    print(" | ".join(row), flush=True)
