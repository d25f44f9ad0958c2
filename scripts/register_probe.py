#!/usr/bin/env python3
"""What page-locking the caller's frame per call would cost (mfx_sample's alternative to staging):
hipHostRegister + hipHostUnregister of a 66 MB pageable numpy frame (touched), and a DMA of 66 MB
from device memory into it while registered. Prints one JSON line."""
import ctypes as C
import json
import time

import numpy as np


def main():
    hip = C.CDLL("libamdhip64.so")
    n = 1920 * 1080 * 4
    frame = np.ones(n)  # touched, pageable
    p = C.c_void_p(frame.ctypes.data)
    nbytes = C.c_size_t(frame.nbytes)
    dev = C.c_void_p()
    assert hip.hipMalloc(C.byref(dev), nbytes) == 0
    reg, unreg, dma = [], [], []
    for _ in range(6):
        t0 = time.perf_counter()
        rc = hip.hipHostRegister(p, nbytes, 0)
        t1 = time.perf_counter()
        assert rc == 0, rc
        assert hip.hipMemcpy(p, dev, nbytes, 2) == 0  # hipMemcpyDeviceToHost
        t2 = time.perf_counter()
        assert hip.hipHostUnregister(p) == 0
        t3 = time.perf_counter()
        reg.append((t1 - t0) * 1e3)
        dma.append((t2 - t1) * 1e3)
        unreg.append((t3 - t2) * 1e3)
    print(json.dumps({"register_ms": [round(x, 3) for x in reg], "dma_ms": [round(x, 3) for x in dma],
                      "unregister_ms": [round(x, 3) for x in unreg], "bytes": frame.nbytes}), flush=True)


if __name__ == "__main__":
    main()
