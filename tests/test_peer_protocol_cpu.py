"""Model of the peer-halo protocol (MAD_OPT_PEER_HALO, csrc/mad_solver.hip Solver::peer_resolve,
mad_kernels.hpp gs_fused3_k<..., PEER> / peer_unpack_k) with ranks as host threads and random
delays: every rank runs the same sequence of sweeps; sweep k stores the rank's edge planes into the
neighbours' mailbox k mod 2 at any moment while it runs (the edge chunks finish early), then counts
itself into the neighbours' counter k mod 2; the next consumer waits until its counters are full,
copies the mailbox out and resets the counters; the next sweep starts after that.  Checked over many
interleavings and 2 / 3 / 5 ranks: every copy sees exactly the neighbour's sweep-k planes (a mailbox
is never overwritten before it was copied out), and no counter ever holds more than one batch (a
reset never loses a signal).  The GPU tests check the kernels; this checks the ordering argument in
DESIGN.md ("Peer halo").  The per-colour levels' push (peer_push_k after the last colour pass, round
5) is the same sequence -- store, count, the neighbour's unpack before the next push -- with the
buffer chosen by a per-level push counter instead of the ping-pong pair's identity."""
import random
import threading

import pytest


class Window:
    def __init__(self):
        self.mb = [[None, None], [None, None]]   # [buffer][side] -> (producer, sweep)
        self.cnt = [[0, 0], [0, 0]]
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)


def run_model(nranks, sweeps, seed):
    rng = random.Random(seed)
    delays = [[rng.random() * 1e-3 for _ in range(4 * sweeps)] for _ in range(nranks)]
    win = [Window() for _ in range(nranks)]
    errors = []

    def rank(r):
        d = iter(delays[r])
        import time
        for k in range(sweeps):
            buf = (k + 1) % 2                      # this sweep's output buffer (ping-pong)
            time.sleep(next(d))                    # the sweep runs; edge chunks finish early
            for nb, side in ((r - 1, 1), (r + 1, 0)):  # bottom edge -> rank-1 (its side 1), top -> rank+1
                if 0 <= nb < nranks:
                    w = win[nb]
                    with w.cv:
                        if w.cnt[buf][side] != 0:
                            errors.append(f"rank {r} sweep {k}: counter [{buf}][{side}] of rank {nb} not reset")
                        if w.mb[buf][side] is not None:
                            errors.append(f"rank {r} sweep {k}: mailbox [{buf}][{side}] of rank {nb} "
                                          f"still holds {w.mb[buf][side]}")
                        w.mb[buf][side] = (r, k)
                        w.cnt[buf][side] += 1
                        w.cv.notify_all()
            time.sleep(next(d))                    # rest of the sweep
            # consumer: peer_resolve for x = buffer `buf` before the next ghost-plane use
            w = win[r]
            need = [s for s, nb in ((0, r - 1), (1, r + 1)) if 0 <= nb < nranks]
            with w.cv:
                if not w.cv.wait_for(lambda: all(w.cnt[buf][s] >= 1 for s in need), timeout=20):
                    errors.append(f"rank {r} sweep {k}: wait timed out")
                    return
                for s in need:
                    nb = r - 1 if s == 0 else r + 1
                    if w.mb[buf][s] != (nb, k):
                        errors.append(f"rank {r} sweep {k}: mailbox [{buf}][{s}] holds {w.mb[buf][s]}, "
                                      f"expected {(nb, k)}")
                    if w.cnt[buf][s] != 1:
                        errors.append(f"rank {r} sweep {k}: counter [{buf}][{s}] = {w.cnt[buf][s]}")
                    w.mb[buf][s] = None            # copied out
                    w.cnt[buf][s] = 0              # the last unpack workgroup resets it
            time.sleep(next(d))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    return errors


@pytest.mark.parametrize("nranks", [2, 3, 5])
@pytest.mark.parametrize("seed", range(6))
def test_peer_halo_protocol_orders_mailboxes(nranks, seed):
    assert run_model(nranks, 40, seed) == []
