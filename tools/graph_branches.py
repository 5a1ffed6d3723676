"""Do two independent launch chains captured as fork/join branches of ONE hipGraph overlap on
MI355X?  (the half-batch fork/join capture of round 4 ended in a segmentation
fault in hipGraphInstantiate; this probe captures the same topology -- the capturing stream
records an event, a side stream waits on it, each stream enqueues its own chain, the capturing
stream waits on the side stream's final event -- with plain C-ABI launches, and times it
against the same two chains captured serially on one stream.)

    python tools/graph_branches.py [launches per chain]

Chains: K dependent l3u_norm_act_fwd launches on a [4, 128, 6^3] tensor (a 6^3-level block
tail, ~5 us in the step) per branch; outputs must be bitwise equal between the two graphs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda:0")
N, C, S = 4, 128, 216
g = torch.Generator().manual_seed(3)
rec = torch.rand(N * C, 8, generator=g).to(dev)
rec[:, 1] = 1.0
rec[:, 2] = 0.5      # scale
rec[:, 3] = 0.01     # shift


def chain(buf):
    """K dependent launches ping-ponging between two buffers: out = lrelu(0.5*(in-mean)+0.01)."""
    a, b = buf
    for i in range(K):
        src, dst = (a, b) if i % 2 == 0 else (b, a)
        nat.call("l3u_norm_act_fwd", src.data_ptr(), C * S, rec.data_ptr(), None, src.data_ptr(),
                 C * S, None, None, 0, dst.data_ptr(), C * S, N, C, S, nat.stream())


def make(seed):
    gg = torch.Generator().manual_seed(seed)
    return [torch.rand(N, C, S, generator=gg).to(dev) for _ in range(2)]


def capture(fork):
    bufs = [make(11), make(12)]   # the same inputs for both graphs
    init = [[t.clone() for t in b] for b in bufs]
    gr = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        chain(bufs[0]); chain(bufs[1])   # warm-up (kernel loading) outside the capture
    torch.cuda.synchronize()
    for b, i0 in zip(bufs, init):
        for t, t0 in zip(b, i0):
            t.copy_(t0)
    torch.cuda.synchronize()
    with torch.cuda.graph(gr):
        if fork:
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)            # fork: event record on cur, wait on side
            chain(bufs[0])
            with torch.cuda.stream(side):
                chain(bufs[1])
            cur.wait_stream(side)            # join before the capture ends
        else:
            chain(bufs[0])
            chain(bufs[1])
    torch.cuda.synchronize()
    return gr, bufs, init


def run(gr, bufs, init, reps):
    for b, i0 in zip(bufs, init):
        for t, t0 in zip(b, i0):
            t.copy_(t0)
    gr.replay()
    torch.cuda.synchronize()
    out = [t.clone() for b in bufs for t in b]
    t0 = time.perf_counter()
    for _ in range(reps):
        gr.replay()
    torch.cuda.synchronize()
    return out, (time.perf_counter() - t0) / reps * 1e6


def main():
    gs, bs, ins = capture(False)
    print("serial graph captured", flush=True)
    gf, bf, inf = capture(True)
    print("fork/join graph captured and instantiated", flush=True)
    o_s, us_s = run(gs, bs, ins, 50)
    o_f, us_f = run(gf, bf, inf, 50)
    same = all(torch.equal(a, b) for a, b in zip(o_s, o_f))
    print(f"{K} launches per chain: serial {us_s:.1f} us/replay ({us_s / (2 * K):.2f} per launch), "
          f"fork/join {us_f:.1f} us/replay ({us_f / (2 * K):.2f} per launch); "
          f"overlap {100 * (1 - us_f / us_s):.0f} %; outputs bitwise equal: {same}", flush=True)
    assert same


if __name__ == "__main__":
    main()
