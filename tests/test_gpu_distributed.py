"""z-slab decomposition on the GPU, rehearsed with the in-process transport
(several ranks as threads on one device; the RCCL path exchanges the same
planes).  Distributed results must be BIT-identical to the single-rank run:
ghost planes carry exactly the neighbour's values and every kernel evaluates
the same arithmetic; only norm partial sums are re-associated across ranks."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

SHAPE = (64, 48, 40)  # (z, y, x): levels (64,48,40) (32,24,20) (16,12,10)
# keep coarse levels distributed down to 2 K voxels per rank on these small shapes (the default,
# MAD_MIN_SLAB_VOXELS, replicates everything below level 0 here): the thin-slab paths under test
DEEP = 2048


def _single(fn, T, **kw):
    import multigridanisotropicdiffusion_amd as M
    s = M.Solver(SHAPE, time_step=0.4, **kw)
    s.set_tensor(T)
    s.setup()
    return fn(None, s)


def _multi(nranks, fn, T, **kw):
    from multigridanisotropicdiffusion_amd import distributed as D

    def body(r, s):
        s.set_tensor(T)
        s.setup()
        return fn(r, s)
    return D.run_local(nranks, body, SHAPE, time_step=0.4, min_slab_voxels=DEEP, **kw)


@pytest.mark.parametrize("nranks", [2, 4])
@pytest.mark.parametrize("smoother,gs_kernel,cycle,options", [(0, 0, 0, 0), (0, 1, 0, 0), (2, 0, 0, 0),
                                                              (0, 3, 0, 0), (0, 3, 2, 0), (0, 3, 0, 2),
                                                              (0, 3, 2, 2), (0, 3, 0, 4), (0, 3, 2, 4)])
@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_sweeps_and_vcycles_bitwise(nranks, smoother, gs_kernel, cycle, options, precision):
    """cycle 2 (SMOOTHER): level-0 records carry b (sync_brec on ghost planes).  gs_kernel 3 forces
    the fused sweep on these small levels, in its default serial rank form (one launch, then the
    exchange) or with options 2 (MAD_OPT_OVERLAP_RANK_SWEEP) in the split form (boundary chunks,
    exchange beside the interior launch), or with options 4 (MAD_OPT_PEER_HALO: the sweep stores its
    edge planes into the neighbours' mailboxes; 2 ranks, where the 32-plane slabs make two z-chunks)."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    T = synth.random_spd(SHAPE, seed=3)
    x = synth.image(SHAPE, seed=1)
    b = synth.image(SHAPE, seed=2)
    sl = D.slabs(SHAPE, nranks)

    def fn(r, s):
        z0, z1 = (0, SHAPE[0]) if r is None else sl[r]
        s.upload(0, M.capi.X, x[z0:z1])
        s.upload(0, M.capi.B, b[z0:z1])
        s.smooth(0, 3)
        a = s.download(0, M.capi.X)
        s.vcycle()
        s.vcycle()
        v = s.download(0, M.capi.X)
        return a, v, s.residual(0)
    kw = dict(smoother=smoother, gs_kernel=gs_kernel, cycle=cycle, options=options,
              precision=M.FP32 if precision == "fp32" else M.FP64)
    ref = _single(fn, T, **kw)
    out = _multi(nranks, fn, T, **kw)
    np.testing.assert_array_equal(np.concatenate([o[0] for o in out]), ref[0])
    np.testing.assert_array_equal(np.concatenate([o[1] for o in out]), ref[1])
    for o in out:
        assert abs(o[2] - ref[2]) <= 1e-12 * ref[2]


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_slab_tensor_setup_is_bitwise(nranks):
    """Each rank sets only the tensor planes it stores (mad_tensor_planes: its slab + 8 ghost
    planes per side) and builds its operators from them, coarse tensor ghost planes exchanged
    hop by hop (8 ranks: 8-plane level-0 slabs, 2-plane level-2 slabs, so ghost regions span
    four neighbours).  Sweeps and V-cycles equal the single-rank run bit for bit; a second
    set_tensor + setup on the same contexts (the next VED iteration's pattern) too."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (64, 40, 36)
    T = synth.random_spd(shape, seed=11)  # (6, z, y, x)
    x = synth.image(shape, seed=12)
    b = synth.image(shape, seed=13)
    sl = D.slabs(shape, nranks)

    def fn(r, s):
        z0, z1 = (0, shape[0]) if r is None else sl[r]
        out = []
        for scale in (1.0, 1.75):  # two setups on one context
            Ts = T * scale
            if r is None:
                s.set_tensor(Ts)
            else:
                lo, hi = s.tensor_planes()
                assert lo == max(z0 - 8, 0) and hi == min(z1 + 8, shape[0])
                s.set_tensor_planes(Ts[:, lo:hi], lo)
            s.setup()
            s.upload(0, M.capi.X, x[z0:z1])
            s.upload(0, M.capi.B, b[z0:z1])
            s.smooth(0, 3)
            s.vcycle()
            out.append(s.download(0, M.capi.X))
        return out

    s = M.Solver(shape, time_step=0.4)
    ref = fn(None, s)
    s.close()
    out = D.run_local(nranks, fn, shape, time_step=0.4, min_slab_voxels=DEEP)
    for q in range(2):
        np.testing.assert_array_equal(np.concatenate([o[q] for o in out]), ref[q])


@pytest.mark.parametrize("nranks", [2, 4])
def test_distributed_filter_run_matches_single(nranks):
    """mad_run on slabs (each rank passes its own slab of the image)."""
    _filter_run(nranks)


@pytest.mark.parametrize("tolerance", [1e-6, 1e-10])
def test_distributed_filter_run_with_peer_halo(tolerance):
    """mad_run with MAD_OPT_PEER_HALO and the fused sweep forced (gs_kernel 3) on 2-rank slabs: the
    peer batches are taken in at every ghost-plane use (norms, descents, interpolations, the next
    time step's casts); at 1e-10 the default precision is FP32_REFINE (fp64 residual, fp32 cycles)."""
    import multigridanisotropicdiffusion_amd as M
    _filter_run(2, tolerance=tolerance, options=M.capi.OPT_PEER_HALO, gs_kernel=3, number_of_steps=2)


def _filter_run(nranks, tolerance=1e-6, **kw):
    from multigridanisotropicdiffusion_amd import distributed as D
    T = synth.ved_form(SHAPE)
    img = (synth.image(SHAPE, seed=5) * 100).astype(np.float32)
    sl = D.slabs(SHAPE, nranks)

    def fn(r, s):
        z0, z1 = (0, SHAPE[0]) if r is None else sl[r]
        out, st = s.run(img[z0:z1], out_dtype=np.float32)
        return out, st
    ref, rst = _single(fn, T, tolerance=tolerance, **kw)
    outs = _multi(nranks, fn, T, tolerance=tolerance, **kw)
    full = np.concatenate([o[0] for o in outs])
    assert np.abs(full - ref).max() <= 1e-5 * np.abs(ref).max()
    assert all(o[1]["total_cycles"] == rst["total_cycles"] for o in outs)


@pytest.mark.parametrize("nranks", [2])
@pytest.mark.parametrize("gs_kernel", [4])
@pytest.mark.parametrize("cycle", [0, 2])
def test_single_launch_slab_sweeps_bitwise(nranks, gs_kernel, cycle):
    """gs_kernel 4 on rank slabs deep enough for two z-chunks per tile column (64 planes
    per rank): the single-launch sweep -- the top chunk marches downward, the edge chunks
    signal their finished edge planes and the communication stream exchanges them while
    the sweep runs.  Results equal the single-rank run bit for bit (sweeps, V-cycles)."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (128, 48, 40)
    T = synth.random_spd(shape, seed=6)
    x = synth.image(shape, seed=7)
    b = synth.image(shape, seed=8)
    sl = D.slabs(shape, nranks)

    def fn(r, s):
        z0, z1 = (0, shape[0]) if r is None else sl[r]
        s.upload(0, M.capi.X, x[z0:z1])
        s.upload(0, M.capi.B, b[z0:z1])
        s.smooth(0, 5)
        a = s.download(0, M.capi.X)
        s.vcycle()
        if r is not None:
            assert "single launch" in s.smooth_kernel_name(0), s.smooth_kernel_name(0)
        return a, s.download(0, M.capi.X)

    def single(_, s):
        return fn(None, s)

    s = M.Solver(shape, time_step=0.4, gs_kernel=gs_kernel, cycle=cycle)
    s.set_tensor(T)
    s.setup()
    ref = single(None, s)

    def body(r, s):
        s.set_tensor(T)
        s.setup()
        return fn(r, s)
    out = D.run_local(nranks, body, shape, time_step=0.4, gs_kernel=gs_kernel, cycle=cycle,
                      min_slab_voxels=DEEP)
    np.testing.assert_array_equal(np.concatenate([o[0] for o in out]), ref[0])
    np.testing.assert_array_equal(np.concatenate([o[1] for o in out]), ref[1])


def test_rccl_transport_selftest():
    """The RCCL path on a one-GPU box: a single-rank communicator runs the solver's halo
    exchange (grouped ncclSend/ncclRecv with this rank as both neighbours), the fp64
    allreduce and the slab allgather (mad_comm_selftest); every byte lands where the
    multi-rank exchange would put its neighbour's planes."""
    import ctypes
    import os
    import multigridanisotropicdiffusion_amd as M
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")  # one node: bootstrap on loopback
    L = M.capi.load()
    err = ctypes.c_double(-1.0)
    rc = L.mad_comm_selftest(0, ctypes.byref(err))
    assert rc == 0, L.mad_last_error(None)
    assert err.value == 0.0


def test_solo_transport_times_one_rank():
    """mad_comm_init_solo (measurement only): one interior rank of a 4-rank decomposition alone
    on the device runs sweeps and graph-replayed V-cycles (every exchange a device copy of the
    same bytes) -- the per-rank timing path of tools/bench_local_split.py --solo."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (128, 64, 64)
    z0, z1 = D.slabs(shape, 4)[2]
    for cyc in (M.SMOOTHER, M.VCYCLE):
        s = M.Solver((z1 - z0,) + shape[1:], time_step=0.1, cycle=cyc, nranks=4, rank=2,
                     global_shape=shape, min_slab_voxels=DEEP)
        s.comm_init_solo()
        s.set_tensor(synth.random_spd(shape, seed=9))
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 3)
        if cyc == M.SMOOTHER:
            dev, kern, n = s.bench_smooth(0, 4)
            assert dev > 0 and n >= 4
        else:
            s.vcycle()
            s.vcycle()
            assert s.bench_vcycle(3) > 0
        assert np.isfinite(s.download(0, M.capi.X)).all()
        s.close()


@pytest.mark.parametrize("cycle,gs_kernel,overlap,nu", [(0, 0, 0, 2), (2, 0, 0, 2), (0, 3, 0, 2), (0, 3, 1, 2),
                                                        (0, 3, 4, 2), (2, 3, 4, 2), (0, 0, 4, 2), (0, 0, 4, 1),
                                                        (0, 0, 4, 3)])
def test_solo_graph_replayed_vcycle_equals_eager(cycle, gs_kernel, overlap, nu):
    """The multi-rank V-cycle replays a captured hipGraph on RCCL / SOLO ranks (host bookkeeping
    of which ghost planes are current decides what the graph re-exchanges).  On the SOLO
    transport (deterministic: every exchange a device copy) the same sequence -- sweeps,
    several V-cycles, an odd sweep count in between (the ping-pong parity flips), more
    V-cycles -- equals the eager execution (mad_desc.options MAD_OPT_EAGER_RANK_VCYCLE) bit for
    bit on every level's x and b; gs_kernel 3 puts the fused rank sweep into the graph, serial
    (the default), split (MAD_OPT_OVERLAP_RANK_SWEEP: a communication-stream branch) or with the
    peer halo (MAD_OPT_PEER_HALO: edge planes into the rank's own stand-in mailboxes, the unpack
    launch waiting on its counters inside the graph); gs_kernel 0 with the peer halo pushes after the
    per-colour sweeps and the descents (the single sweep in between flips level 0's mailbox parity,
    which the graph is keyed on: it is re-captured); nu = 1 / 3 sweeps per level (a cycle pushes 2 nu
    batches per level, so a replay leaves the parity where the capture found it)."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (128, 64, 64)
    z0, z1 = D.slabs(shape, 4)[2]
    out = {}
    base = {0: 0, 1: M.capi.OPT_OVERLAP_RANK_SWEEP, 4: M.capi.OPT_PEER_HALO}[overlap]
    for opt in (0, M.capi.OPT_EAGER_RANK_VCYCLE):
        s = M.Solver((z1 - z0,) + shape[1:], time_step=0.3, cycle=cycle, nranks=4, rank=2,
                     global_shape=shape, min_slab_voxels=DEEP, options=opt | base, gs_kernel=gs_kernel,
                     iterations_per_grid=nu)
        s.comm_init_solo()
        s.synth_tensor(kind=0, seed=9)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 4)
        s.smooth(0, 2)
        for _ in range(3):
            s.vcycle()
        s.smooth(0, 1)
        for _ in range(2):
            s.vcycle()
        out[opt] = [(s.download(l, M.capi.X), s.download(l, M.capi.B))
                    for l in range(s.num_levels)]
        s.close()
    a, b = out[0], out[M.capi.OPT_EAGER_RANK_VCYCLE]
    for l, ((xa, ba), (xb, bb)) in enumerate(zip(a, b)):
        assert np.isfinite(xa).all()
        np.testing.assert_array_equal(xa, xb, err_msg=f"x, level {l}")
        np.testing.assert_array_equal(ba, bb, err_msg=f"b, level {l}")


@pytest.mark.parametrize("cycle,gs_kernel,options", [(0, 0, 0), (0, 3, 0), (2, 3, 0), (0, 3, 4), (0, 0, 4)])
def test_rccl_solo_equals_solo(cycle, gs_kernel, options):
    """mad_comm_init_rccl_solo moves SOLO's bytes through RCCL (a single-rank communicator, every
    grouped exchange ncclSend / ncclRecv pairs to itself, inside the captured V-cycle graph too):
    the same sequence -- partitioned setup (hop-by-hop tensor ghost planes), sweeps, graph-replayed
    V-cycles, an odd sweep count, more V-cycles -- gives SOLO's result bit for bit on every level."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (128, 64, 64)
    z0, z1 = D.slabs(shape, 4)[2]
    out = {}
    for mode in ("solo", "rccl"):
        s = M.Solver((z1 - z0,) + shape[1:], time_step=0.3, cycle=cycle, nranks=4, rank=2,
                     global_shape=shape, min_slab_voxels=DEEP, gs_kernel=gs_kernel, options=options)
        if mode == "solo":
            s.comm_init_solo()
        else:
            s.comm_init_rccl_solo()
        s.synth_tensor(kind=0, seed=9)
        s.setup()
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 4)
        s.smooth(0, 2)
        for _ in range(3):
            s.vcycle()
        s.smooth(0, 1)
        for _ in range(2):
            s.vcycle()
        out[mode] = [(s.download(l, M.capi.X), s.download(l, M.capi.B)) for l in range(s.num_levels)]
        s.close()
    for l, ((xa, ba), (xb, bb)) in enumerate(zip(out["solo"], out["rccl"])):
        assert np.isfinite(xa).all()
        np.testing.assert_array_equal(xa, xb, err_msg=f"x, level {l}")
        np.testing.assert_array_equal(ba, bb, err_msg=f"b, level {l}")


@pytest.mark.parametrize("rank", [0, 3])
def test_solo_peer_halo_end_ranks(rank):
    """MAD_OPT_PEER_HALO on a rank at either end of the decomposition (one neighbour): on the SOLO
    transport its edge chunk fills its own stand-in mailbox of the side it has, so every unpack's
    wait is met -- sweeps, graph-replayed V-cycles and the download's peer check finish (a wait
    that timed out would raise there)."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (128, 64, 64)
    z0, z1 = D.slabs(shape, 4)[rank]
    for cycle in (0, 2):
        s = M.Solver((z1 - z0,) + shape[1:], time_step=0.3, cycle=cycle, nranks=4, rank=rank,
                     global_shape=shape, min_slab_voxels=DEEP, options=M.capi.OPT_PEER_HALO, gs_kernel=3)
        s.comm_init_solo()
        s.synth_tensor(kind=0, seed=9)
        s.setup()
        assert "peer halo" in s.smooth_kernel_name(0)
        s.synth_level(0, M.capi.B, 3)
        s.synth_level(0, M.capi.X, 4)
        s.smooth(0, 3)
        for _ in range(3):
            s.vcycle()
        assert np.isfinite(s.download(0, M.capi.X)).all()
        s.close()


@pytest.mark.parametrize("nranks", [2, 4])
@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_per_colour_peer_halo_bitwise(nranks, precision):
    """MAD_OPT_PEER_HALO with the default kernels (round 5): on these small levels every distributed
    level sweeps colour by colour, so each sweep pushes its edge planes into the neighbours' mailboxes
    after its last colour pass (peer_push_k), each descent pushes the coarse level's new b, and the
    next consumer unpacks them -- no exchange.  The option must engage on every distributed level of
    at least GHOST planes (the kernel name says so), and sweeps, V-cycles and the residual equal the
    single-rank run bit for bit."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    T = synth.random_spd(SHAPE, seed=5)
    x = synth.image(SHAPE, seed=6)
    b = synth.image(SHAPE, seed=7)
    sl = D.slabs(SHAPE, nranks)
    global_nz = [SHAPE[0] >> l for l in range(8)]

    def fn(r, s):
        z0, z1 = (0, SHAPE[0]) if r is None else sl[r]
        peer = []
        if r is not None:
            for l in range(s.num_levels):
                nz = s.level_info(l)["shape"][0]
                name = s.smooth_kernel_name(l)
                if nz < global_nz[l] and nz >= 4:  # a rank slab of >= GHOST planes
                    assert "gs_color_k" in name and "peer halo" in name, (l, name)
                    peer.append(l)
        s.upload(0, M.capi.X, x[z0:z1])
        s.upload(0, M.capi.B, b[z0:z1])
        s.smooth(0, 3)
        a = s.download(0, M.capi.X)
        for _ in range(3):
            s.vcycle()
        v = s.download(0, M.capi.X)
        return a, v, s.residual(0), peer
    kw = dict(options=M.capi.OPT_PEER_HALO, precision=M.FP32 if precision == "fp32" else M.FP64)
    ref = _single(fn, T, **kw)
    out = _multi(nranks, fn, T, **kw)
    assert all(0 in o[3] and len(o[3]) >= 2 for o in out), [o[3] for o in out]
    np.testing.assert_array_equal(np.concatenate([o[0] for o in out]), ref[0])
    np.testing.assert_array_equal(np.concatenate([o[1] for o in out]), ref[1])
    for o in out:
        assert abs(o[2] - ref[2]) <= 1e-12 * ref[2]


@pytest.mark.parametrize("cycle", [0, 1, 2])       # VCYCLE, FMG, SMOOTHER (20 sweeps, unconverged)
@pytest.mark.parametrize("precision", [1, 2])      # FP64, FP32_REFINE
@pytest.mark.parametrize("peer", [False, True])
@pytest.mark.parametrize("in_dtype", [np.float64, np.float32])
@pytest.mark.parametrize("nranks", [2, 4])
def test_filter_run_rank_slabs_bitwise(cycle, precision, peer, in_dtype, nranks):
    """mad_run on 2 / 4 in-process rank slabs over two time steps, every CycleType x
    precision x halo form x input type (fp32: the refine mode's exactly-fp32 rhs): the output equals
    the single-rank run bit for bit, with the same cycle counts.  FMG + peer halo + FP32_REFINE
    once ended 5e-12 away (a peer batch from the previous step landing on the ghost planes FMG's
    interpolation had written; profiles/r05_fmg_peer_fix.log)."""
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    shape = (64, 48, 40)
    T = synth.ved_form(shape)
    img = (synth.image(shape, seed=5) * 100).astype(in_dtype)
    sl = D.slabs(shape, nranks)
    kw = dict(time_step=0.4, tolerance=1e-10, precision=precision, number_of_steps=2, cycle=cycle,
              options=M.capi.OPT_PEER_HALO if peer else 0, max_cycles=20 if cycle == 2 else 100)
    s = M.Solver(shape, **kw)
    s.set_tensor(T)
    ref, rst = s.run(img, out_dtype=np.float64)
    s.close()

    def body(r, s):
        s.set_tensor(T)
        s.setup()
        z0, z1 = sl[r]
        return s.run(img[z0:z1], out_dtype=np.float64)
    outs = D.run_local(nranks, body, shape, **kw)
    assert cycle == 2 or rst["last_relres"] <= 1e-10
    np.testing.assert_array_equal(np.concatenate([o[0] for o in outs]), ref)
    assert all(list(o[1]["step_cycles"]) == list(rst["step_cycles"]) for o in outs)
