import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/tests')
import multigridanisotropicdiffusion_amd as M
import ved_oracle as VO
SP = (0.3125, 0.3125, 0.5)
rng = np.random.default_rng(11)
shape = (22, 26, 30)
img = rng.normal(50.0, 20.0, size=shape)
for sigma in (0.3, 0.775, 2.0):
    v = M.VED(shape, SP, precision=M.FP32, hessian="recursive")
    H = v.hessian(img, sigma)
    ref = VO.hessian(img, SP, sigma, "recursive")
    print(sigma, ["%.2e" % (np.abs(H[q] - ref[..., q]).max() / np.abs(ref[..., q]).max()) for q in range(6)])
