#!/usr/bin/env python3
"""SearchForInitialization walk statistics on the C2 bench data, from a
library built with -DORB_SFI_COUNT (variants/lib_sfic.so copied over the
product library): rounds of the speculative walk, partial rounds, rescans."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from orb_slam3_vio_fixes_amd import capi, orb, synth
    W, H, B = 752, 480, 256
    frames = torch.from_numpy(synth.sequence(W, H, B, config=2)).cuda()
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    k, d, n, m, cap = ex.extract_batch_device(frames, (0, 1000))
    L = capi.lib()
    if not hasattr(L, "orbm_debug_sfi_counts"):   # product library: timing only
        L.orbm_debug_sfi_counts = lambda *a: 0
    else:
        L.orbm_debug_sfi_counts.argtypes = [C.c_void_p, C.c_int]
    out = np.zeros(16, np.uint64)
    L.orbm_debug_sfi_counts(out.ctypes.data, 1)
    matches = torch.empty((B - 1, cap), dtype=torch.int32, device="cuda")
    nm = torch.empty(B - 1, dtype=torch.int32, device="cuda")
    def call():
        rc = L.orbm_search_for_initialization_batch_device(
            B, k.data_ptr(), d.data_ptr(), n.data_ptr(), cap, 0.0, float(W), 0.0, float(H),
            float(np.float32(64) / np.float32(W)), float(np.float32(48) / np.float32(H)), 100, 0.9, 1,
            matches.data_ptr(), nm.data_ptr(), torch.cuda.current_stream().cuda_stream)
        capi.check(rc, "SearchForInitialization batch")
    call()   # warm-up (scratch, code objects)
    torch.cuda.synchronize()
    L.orbm_debug_sfi_counts(out.ctypes.data, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call()
    e1.record()
    torch.cuda.synchronize()
    print(f"batch call alone (top-K + resolve, {B - 1} pairs): {e0.elapsed_time(e1) * 1e3:.1f} us")
    L.orbm_debug_sfi_counts(out.ctypes.data, 0)
    pairs = B - 1
    print(f"pairs {pairs}: queries {out[3] / pairs:.1f}, rounds {out[0] / pairs:.1f}, continuations "
          f"{out[1] / pairs:.1f}, rescans {out[2] / pairs:.2f}, claims {out[4] / pairs:.1f} per pair; "
          f"nmatches mean {nm.float().mean().item():.1f}")
    names = ["decide", "conflict scan", "commit", "state update", "rescan", "run advance", "prologue", "block"]
    print("kcycles per pair: " + ", ".join(f"{nme} {out[8 + i] / pairs / 1e3:.1f}" for i, nme in enumerate(names)))


if __name__ == "__main__":
    main()
