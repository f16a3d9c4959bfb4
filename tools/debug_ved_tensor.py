"""Where does the fp32 VED tensor differ most from the numpy oracle on the reference's
ved_test volume (itkVEDTest_GS parameters)?  Prints the worst voxels with their responses.
    python tools/debug_ved_tensor.py"""
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
    img, info = mhd.read_mhd(os.path.join(ROOT, "tests", "golden", "ved_test.mhd"))
    sp = tuple(info["spacing"])
    kw = dict(alpha=0.5, beta=0.5, gamma=5.0, epsilon=0.01, sensitivity=10.0, omega=1.5)
    img = img.astype(np.float64)
    Tr, rr = VO.ved_tensor(img, sp, **kw)
    for prec in ("FP32", "FP64"):
        v = M.VED(img.shape, sp, precision=getattr(M, prec), **kw)
        T, resp = v.tensor(img)
        d = np.abs(T - Tr).max(axis=0)
        idx = np.argsort(d.ravel())[::-1][:5]
        print(prec, "max |T - Tr| =", d.max(), " max |resp - rr| =", np.abs(resp - rr).max())
        for q in idx:
            z, y, x = np.unravel_index(q, d.shape)
            print(f"  voxel {(z, y, x)}: dT {d[z, y, x]:.3e} resp gpu {resp[z, y, x]:.6e} "
                  f"oracle {rr[z, y, x]:.6e} T gpu {np.round(T[:, z, y, x], 5)} "
                  f"oracle {np.round(Tr[:, z, y, x], 5)}")


if __name__ == "__main__":
    main()
