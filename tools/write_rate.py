#!/usr/bin/env python3
"""Host file-write rate vs writer threads (the create-streaming write stage): N bytes from one buffer into a fresh
file (O_TRUNC + ftruncate, as streaming.create_streaming_array does) with pwrite in k threads over disjoint ranges.
Usage: write_rate.py DIR [GB]"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def main():
    d = sys.argv[1]
    nbytes = int(float(sys.argv[2] if len(sys.argv) > 2 else 3.0) * (1 << 30))
    buf = np.ones(nbytes, dtype=np.uint8)
    mv = memoryview(buf)
    path = os.path.join(d, f"write_rate_{os.getpid()}.bin")
    try:
        for k in (1, 4, 8, 16, 32, 8):
            for chunk_mb in (8, 64):
                fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
                os.ftruncate(fd, nbytes)
                ch = chunk_mb << 20
                pieces = [(o, min(ch, nbytes - o)) for o in range(0, nbytes, ch)]

                def run(t):
                    for o, n in pieces[t::k]:
                        done = 0
                        while done < n:
                            done += os.pwrite(fd, mv[o + done:o + n], o + done)
                t0 = time.perf_counter()
                with ThreadPoolExecutor(k) as ex:
                    list(ex.map(run, range(k)))
                dt = time.perf_counter() - t0
                os.close(fd)
                print(f"threads {k:2d} chunk {chunk_mb:3d} MB: {nbytes / dt / 1e9:6.2f} GB/s ({dt:.3f} s)", flush=True)
                os.unlink(path)
    finally:
        if os.path.exists(path):
            os.unlink(path)


if __name__ == "__main__":
    main()
