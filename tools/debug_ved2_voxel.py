"""One voxel of the fp32 VED tensor against the oracle on ved_test_2 (itkVEDTest_GS parameters):
the GPU tensor (fp32 / fp64 modes), the oracle's, every scale's response and eigenvalues there.
    python tools/debug_ved2_voxel.py [z y x]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import mhd
    import ved_oracle as VO
    img, info = mhd.read_mhd(os.path.join(ROOT, "tests", "golden", "ved_test_2.mhd"))
    sp = tuple(info["spacing"])
    kw = dict(alpha=0.5, beta=0.5, gamma=5.0, epsilon=0.01, sensitivity=10.0, omega=1.5)
    x = img.astype(np.float64)
    Tr, rr = VO.ved_tensor(x, sp, **kw)
    Ts = {}
    for prec in ("FP32", "FP64"):
        v = M.VED(img.shape, sp, precision=getattr(M, prec), **kw)
        Ts[prec] = v.tensor(img)
        v.close()
    d = np.abs(Ts["FP32"][0] - Tr).max(axis=0)
    pts = [tuple(int(a) for a in sys.argv[1:4])] if len(sys.argv) > 3 else \
        [np.unravel_index(q, d.shape) for q in np.argsort(d.ravel())[::-1][:4]]
    for (z, y, xx) in pts:
        print(f"voxel {(z, y, xx)}: dT32 {d[z, y, xx]:.3e} dT64 "
              f"{np.abs(Ts['FP64'][0][:, z, y, xx] - Tr[:, z, y, xx]).max():.3e}")
        print("  T fp32  ", np.round(Ts["FP32"][0][:, z, y, xx], 6), "resp", Ts["FP32"][1][z, y, xx])
        print("  T fp64  ", np.round(Ts["FP64"][0][:, z, y, xx], 6), "resp", Ts["FP64"][1][z, y, xx])
        print("  T oracle", np.round(Tr[:, z, y, xx], 6), "resp", rr[z, y, xx])
        for s in VO.DEFAULTS["scales"]:
            H = VO.hessian(x, sp, s)[z, y, xx]
            A = np.array([[H[0], H[1], H[2]], [H[1], H[3], H[4]], [H[2], H[4], H[5]]])
            w, vv = np.linalg.eigh(A)
            ves = VO.vesselness(VO.sort_by_magnitude(w[None]), kw["alpha"], kw["beta"], kw["gamma"])[0]
            print(f"  scale {s}: eig {w} ves {ves:.9e} v3 {np.round(vv[:, 2], 5)}")


if __name__ == "__main__":
    main()
