"""Stage-by-stage parity probe of the HIP extractor against the CPU oracle
(run on the GPU box).  Prints the first divergence of each stage."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from orb_slam3_vio_fixes_amd import orb, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def cmp_stage(name, a, b):
    ok = True
    for l, (x, y) in enumerate(zip(a, b)):
        if len(x) != len(y):
            print(f"  {name} L{l}: count {len(x)} vs oracle {len(y)}")
            ok = False
            continue
        fx = np.stack([x["x"], x["y"], x["response"]], 1)
        fy = np.stack([y["x"], y["y"], y["response"]], 1)
        bad = np.nonzero(np.any(fx != fy, 1))[0]
        if len(bad):
            i = bad[0]
            print(f"  {name} L{l}: {len(bad)} diffs, first #{i}: {fx[i]} vs {fy[i]}")
            ok = False
    print(f"{name}: {'OK' if ok else 'MISMATCH'}")
    return ok


def main(n=3, w=752, h=480, nfeat=1000, lap=(0, 1000)):
    ex = orb.ORBextractor(nfeat, 1.2, 8, 20, 7)
    ref = O.OracleExtractor(nfeat, 1.2, 8, 20, 7)
    allok = True
    for i in range(n):
        img = synth.image(w, h, synth.frame_seed(2, i))
        k, d, m = ex(img, None, lap)
        rk, rd, rm = ref(img, lap)
        print(f"frame {i}: n={len(k)} oracle n={len(rk)} mono={m}/{rm}")
        pg = ex.mvImagePyramid
        for l in range(8):
            po = ref.level(l)
            if not np.array_equal(pg[l], po):
                diff = np.argwhere(pg[l] != po)
                print(f"  pyramid L{l}: {len(diff)} px differ, first {diff[0]} {pg[l][tuple(diff[0])]} vs {po[tuple(diff[0])]}")
                allok = False
        allok &= cmp_stage("candidates", ex.debug_stage(0), ref.stage(0))
        allok &= cmp_stage("quadtree", ex.debug_stage(1), ref.stage(1))
        if len(k) == len(rk):
            kb = k.view(np.uint8).reshape(len(k), 28)
            rb = rk.view(np.uint8).reshape(len(rk), 28)
            badk = np.nonzero(np.any(kb != rb, 1))[0]
            badd = np.nonzero(np.any(d != rd, 1))[0]
            print(f"  keypoint rows differing: {len(badk)}; descriptor rows differing: {len(badd)}")
            if len(badk):
                print("   first kp", k[badk[0]], rk[badk[0]])
            if len(badd):
                print("   first desc row", badd[0], d[badd[0]][:8], rd[badd[0]][:8], k[badd[0]])
            allok &= len(badk) == 0 and len(badd) == 0 and m == rm
        else:
            allok = False
    print("ALL OK" if allok else "PARITY FAIL")
    return allok


if __name__ == "__main__":
    ok = main()
    ok &= main(n=1, w=512, h=512, nfeat=1500, lap=(0, 511))
    ok &= main(n=1, w=1920, h=1080, nfeat=5000, lap=(0, 1000))
    sys.exit(0 if ok else 1)
