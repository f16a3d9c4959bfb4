"""ISA evidence for the peer halo's memory ordering: compiles
csrc/mad_solver.hip for gfx950 with --save-temps into a scratch directory and prints, for the
producer (gs_fused3_k<float, FULL, ..., PEER = true, ...>, peer_push_k, peer_ping_k) and the consumer
(peer_unpack_k, peer_pong_k), the instructions that carry the protocol: the mailbox stores and
their cache-policy bits, the s_waitcnt before the counter atomic, the atomic's scope bits, and
the system-scope acquire (load sc0 sc1 + buffer_inv sc0 sc1) before the mailbox reads.
    python tools/peer_isa.py [scratch_dir]  > profiles/r05_peer_isa.txt"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "multigridanisotropicdiffusion_amd", "csrc", "mad_solver.hip")

KEEP = re.compile(r"(buffer_store|global_store|global_atomic|buffer_atomic|flat_atomic|s_waitcnt vmcnt\(0\)|"
                  r"buffer_inv|buffer_wbl2|global_load_dword\S* .*sc[01]|s_barrier|s_sleep|s_memrealtime)")


def functions(asm):
    """{symbol: [lines]} of the device assembly."""
    out, cur = {}, None
    for ln in asm.splitlines():
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            if ln.startswith(".Lfunc_end"):
                cur = None
                continue
            out[cur].append(ln)
    return out


def excerpt(name, lines, limit=90):
    print(f"\n### {name}\n")
    body = [ln for ln in lines if ln.strip() and not ln.lstrip().startswith((";", ".loc", ".file", ".cfi"))]
    keep = [i for i, ln in enumerate(body) if KEEP.search(ln)]
    shown, last = 0, -10
    for i in keep:
        lo = max(i - 2, last + 1)
        if lo > last + 1 and shown:
            print("\t...")
        for j in range(lo, i + 1):
            print(body[j])
            shown += 1
        last = i
        if shown >= limit:
            print("\t... (truncated)")
            break
    s = "\n".join(body)
    print(f"\n    counts: buffer_store {s.count('buffer_store')}, global_atomic {s.count('global_atomic')}, "
          f"buffer_inv {s.count('buffer_inv')}, buffer_wbl2 {s.count('buffer_wbl2')}")


def main():
    work = sys.argv[1] if len(sys.argv) > 1 else "/tmp/mad_isa"
    os.makedirs(work, exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-Wno-unused-function", "--save-temps", "-c", "-o", os.path.join(work, "mad.o"), SRC],
                          cwd=work)
    asm = open(os.path.join(work, "mad_solver-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    fn = functions(asm)
    want = [
        ("producer: the production fp32 full-tensor rank sweep, V-cycle layout (BREC 0, PEER 1, BL 1)",
         "_ZN3mad11gs_fused3_kIfLi3ELi64ELi32ELi1024ELi4ELi2ELb0ELb1ELb1ELb0E"),
        ("producer: the same sweep in the SMOOTHER layout (BREC 1, PEER 1)",
         "_ZN3mad11gs_fused3_kIfLi3ELi64ELi32ELi1024ELi4ELi2ELb1ELb1ELb0ELb0E"),
        ("producer: per-colour levels' edge planes and the descents' coarse b (round 5) peer_push_k<float>",
         "_ZN3mad11peer_push_kIfE"),
        ("setup self-test producer peer_ping_k<float>", "_ZN3mad11peer_ping_kIfE"),
        ("consumer peer_unpack_k", "_ZN3mad13peer_unpack_k"),
        ("setup self-test consumer peer_pong_k<float>", "_ZN3mad11peer_pong_kIfE"),
    ]
    print("# Peer-halo ISA excerpts (gfx950, hipcc -O3 --save-temps of csrc/mad_solver.hip)")
    for title, prefix in want:
        names = [n for n in fn if n.startswith(prefix)]
        if not names:
            print(f"\n### {title}: NOT FOUND ({prefix})")
            continue
        excerpt(f"{title}\n`{names[0]}`", fn[names[0]])


if __name__ == "__main__":
    main()
