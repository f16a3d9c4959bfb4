"""Generate the committed golden fixtures (run from the repo root, CPU only):

    python tests/golden/make_golden.py

Inputs
  lena_512_u8.npy   the reference's whole test/test_data/lena.jpg (512x512, grayscale JPEG),
                    decoded once with PIL; the reference reads it as unsigned char
                    (test/itk2DDiffusionTest_GS.cxx:21-42) -- the input of the nine ctest
                    registrations (tests/test_gpu_registrations.py)
  lena_256_u8.npy   centre 256x256 crop of it (BASELINE config C1)
  ved_crop_i16.npy  35x39x35 crop (z,y,x) of test/test_data/ved_test.zraw (zlib,
                    int16, DimSize 69 77 69, spacing .3125 .3125 .5)
  ved2_crop_i16.npy 55x52x54 centre crop (z,y,x) of test/test_data/ved_test_2.zraw (zlib,
                    int16, DimSize 134 140 119, spacing .330017): its hierarchy coarsens
                    CCV -> VCC -> CVC (x,y,z), the first three of the full volume's
                    CCV -> VCC -> CVC -> VCV
  (python tests/golden/make_golden.py lena512 writes only lena_512_u8.npy,
   python tests/golden/make_golden.py ved2   regenerates only the ved_test_2 fixtures,
   python tests/golden/make_golden.py lena64 only the fp64 lena solutions lena_c1_f64.npz)
Expected outputs come from the fp64 oracle (oracle/), which restates the
reference line by line.  PARITY UNPINNED: the reference has no golden vectors
of its own and cannot be built here, so these pin the GPU path to the oracle
and the oracle to itself (regression), not to reference-produced numbers.
"""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as O  # noqa: E402
import synth  # noqa: E402

REF = "/root/reference/test/test_data"


def make_inputs():
    from PIL import Image
    lena = np.asarray(Image.open(os.path.join(REF, "lena.jpg")).convert("L"))
    np.save(os.path.join(HERE, "lena_512_u8.npy"), np.ascontiguousarray(lena))
    c0 = (lena.shape[0] - 256) // 2
    np.save(os.path.join(HERE, "lena_256_u8.npy"), np.ascontiguousarray(lena[c0:c0 + 256, c0:c0 + 256]))
    raw = zlib.decompress(open(os.path.join(REF, "ved_test.zraw"), "rb").read())
    ved = np.frombuffer(raw, dtype="<i2").reshape(69, 77, 69)  # (z, y, x)
    np.save(os.path.join(HERE, "ved_crop_i16.npy"), np.ascontiguousarray(ved[17:52, 19:58, 17:52]))
    make_ved2_input()


VED2_SPACING = (0.330017, 0.330017, 0.330017)


def make_ved2_input():
    raw = zlib.decompress(open(os.path.join(REF, "ved_test_2.zraw"), "rb").read())
    v2 = np.frombuffer(raw, dtype="<i2").reshape(119, 140, 134)  # (z, y, x)
    np.save(os.path.join(HERE, "ved2_crop_i16.npy"), np.ascontiguousarray(v2[32:87, 44:96, 40:94]))


def ved2_mad():
    """itkVEDTest_GS MAD parameters (nu 3, dt 0.1, 4 steps, tolerance 1e-10, lexicographic GS;
    test/itkVEDTest_GS.cxx:61,84-88) on the ved_test_2 crop with a VED-form tensor."""
    v2 = np.load(os.path.join(HERE, "ved2_crop_i16.npy")).astype(np.float64)
    T = synth.ved_form(v2.shape)
    o = O.Oracle(v2.shape, VED2_SPACING, T, 0.1)
    out, c, rr = o.run(v2, cycle=O.VCYCLE, smoother=O.GS_LEX, tolerance=1e-10,
                       iterations_per_grid=3, number_of_steps=4)
    print("ved2", [lv["shape"] for lv in o.levels], c, rr)
    np.savez_compressed(os.path.join(HERE, "ved2_mad.npz"), out=out, cycles=np.array(c),
                        relres=np.array(rr), spacing=np.array(VED2_SPACING))


# per-kernel cases: (name, shape, spacing x-first, tensor maker, dt)
KERNEL_CASES = [
    ("k2d_cell", (24, 18), (1.0, 0.5), lambda s: synth.random_spd(s, seed=3), 0.3),
    ("k2d_vert", (25, 19), (0.8, 1.1), lambda s: synth.random_spd(s, seed=5), 0.2),
    ("k3d_vert", (13, 17, 11), (0.7, 1.0, 1.3), lambda s: synth.random_spd(s, seed=7), 0.3),
    ("k3d_cell", (16, 16, 16), (1.0, 1.0, 1.0), lambda s: synth.random_spd(s, seed=9), 0.5),
    ("k3d_mixed", (12, 14, 13), (1.0, 1.0, 1.0), lambda s: synth.random_spd(s, seed=11), 0.4),
    ("k3d_diag", (16, 14, 18), (1.0, 1.0, 1.0), lambda s: synth.random_spd(s, seed=13, offdiag=False), 0.4),
    ("k3d_iso", (16, 16, 16), (1.0, 1.0, 1.0), lambda s: synth.isotropic(s, seed=2), 0.5),
    ("k3d_deep", (24, 26, 28), (1.0, 0.9, 1.2), lambda s: synth.random_spd(s, seed=15), 0.6),
    ("k2d_deep", (48, 40), (1.0, 1.0), lambda s: synth.random_spd(s, seed=17), 0.8),
]


def kernel_case(name, shape, spacing, tmaker, dt):
    T = tmaker(shape)
    o = O.Oracle(shape, spacing, T, dt)
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    x = rng.random(shape)
    b = rng.random(shape)
    d = dict(shape=np.array(shape), spacing=np.array(spacing), dt=np.array(dt), tensor=T, x=x, b=b)
    diag = name.endswith("diag") or name.endswith("iso")
    d["wj"] = o.wj(0, x, b)
    d["residual"] = o.residual(0, x, b)
    d["gs_lex"] = o.gs_lex(0, x, b)
    d["gs_color"] = o.gs_color(0, x, b, ncolors=2 if diag else 4)
    if o.num_levels > 1:
        d["restrict"] = o.restrict(0, d["residual"])
        xc = rng.random(o.shape_at(1))
        d["xc"] = xc
        d["interp"] = o.interpolate(0, xc)
    L = o.num_levels - 1
    bc = rng.random(o.shape_at(L))
    d["bc"] = bc
    d["coarse_solve"] = o.direct_solve(bc)
    d["vcycle_wj"] = o.vcycle(x, b, smoother=O.WJ)
    d["vcycle_gs_color"] = o.vcycle(x, b, smoother=O.GS_COLOR, ncolors=2 if diag else 4)
    d["vcycle_gs_lex"] = o.vcycle(x, b, smoother=O.GS_LEX)
    d["fmg_wj"] = o.fmg(b, smoother=O.WJ)
    out, cyc, rr = o.run(b, tolerance=1e-11, smoother=O.GS_LEX)
    d["run_gs_lex"] = out
    d["run_gs_lex_cycles"] = np.array(cyc)
    return d


def lena_f64():
    """C1 (itk2DDiffusionTest_{GS,WJ}) oracle solutions in fp64 (lena_c1.npz keeps them in
    fp32): the references of the MAD_FP32_REFINE tests, which resolve 1e-9."""
    lena = np.load(os.path.join(HERE, "lena_256_u8.npy")).astype(np.float64)
    T = synth.constant(lena.shape, (50.0, 0.0, 30.0))
    o = O.Oracle(lena.shape, (1.0, 1.0), T, 0.1)
    res = {}
    for sm, tag in ((O.WJ, "wj"), (O.GS_LEX, "gs")):
        for cyc, ctag in ((O.VCYCLE, "v"), (O.FMG, "fmg")):
            out, c, rr = o.run(lena, cycle=cyc, smoother=sm, tolerance=1e-10, iterations_per_grid=2)
            res[f"{tag}_{ctag}"] = out
            res[f"{tag}_{ctag}_cycles"] = np.array(c)
            res[f"{tag}_{ctag}_relres"] = np.array(rr)
    np.savez_compressed(os.path.join(HERE, "lena_c1_f64.npz"), **res)


def make_lena512():
    from PIL import Image
    lena = np.asarray(Image.open(os.path.join(REF, "lena.jpg")).convert("L"))
    assert lena.shape == (512, 512) and lena.dtype == np.uint8
    np.save(os.path.join(HERE, "lena_512_u8.npy"), np.ascontiguousarray(lena))


def main():
    if sys.argv[1:] == ["lena512"]:
        make_lena512()
        return
    if sys.argv[1:] == ["lena64"]:
        lena_f64()
        return
    if sys.argv[1:] == ["ved2"]:
        if os.path.isdir(REF):
            make_ved2_input()
        ved2_mad()
        return
    if os.path.isdir(REF):
        make_inputs()
    for case in KERNEL_CASES:
        d = kernel_case(*case)
        np.savez_compressed(os.path.join(HERE, case[0] + ".npz"), **d)
        print(case[0], "levels", O.Oracle(case[1], case[2], case[3](case[1]), case[4]).num_levels)
    # C1 config (itk2DDiffusionTest_WJ): lena 256^2, M = [[50,0],[0,30]], dt 0.1, nu 2
    lena = np.load(os.path.join(HERE, "lena_256_u8.npy")).astype(np.float64)
    T = synth.constant(lena.shape, (50.0, 0.0, 30.0))
    o = O.Oracle(lena.shape, (1.0, 1.0), T, 0.1)
    res = {}
    for sm, tag in ((O.WJ, "wj"), (O.GS_LEX, "gs")):
        for cyc, ctag in ((O.VCYCLE, "v"), (O.FMG, "fmg")):
            out, c, rr = o.run(lena, cycle=cyc, smoother=sm, tolerance=1e-10, iterations_per_grid=2)
            res[f"{tag}_{ctag}"] = out.astype(np.float32)
            res[f"{tag}_{ctag}_cycles"] = np.array(c)
            print("lena", tag, ctag, c, rr)
    np.savez_compressed(os.path.join(HERE, "lena_c1.npz"), **res)
    lena_f64()
    # VED-test MAD parameters on the ved crop with a VED-form tensor:
    # nu 3, dt 0.1, 4 steps (test/itkVEDTest_GS.cxx:61,84-88), spacing .3125 .3125 .5
    ved = np.load(os.path.join(HERE, "ved_crop_i16.npy")).astype(np.float64)
    T = synth.ved_form(ved.shape)
    sp = (0.3125, 0.3125, 0.5)
    o = O.Oracle(ved.shape, sp, T, 0.1)
    out, c, rr = o.run(ved, cycle=O.VCYCLE, smoother=O.GS_LEX, tolerance=1e-10,
                       iterations_per_grid=3, number_of_steps=4)
    print("ved", c, rr)
    np.savez_compressed(os.path.join(HERE, "ved_mad.npz"), out=out, cycles=np.array(c),
                        spacing=np.array(sp))
    ved2_mad()


if __name__ == "__main__":
    main()
