"""Where a training step's wall time goes, from a rocprofv3 --kernel-trace CSV: one steady-state
step (between the last two launches of the fused BertAdam update), split into phases by marker
kernels (trunk forward, encoder forward, encoder backward, trunk backward, optimizer), with per
phase the wall time, the GPU-busy time (union of all kernels' intervals), the time with two or
more kernels running (streams overlapping) and the main stream's own busy time.

  python tools/step_timeline.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", r["Queue_Id"]))
         for r in rows]
    k.sort()
    adam = [s for s, e, n, q in k if "adam_update_kernel" in n]
    t0, t1 = adam[-2], adam[-1]
    step = [x for x in k if t0 <= x[0] < t1]
    # phase markers (first occurrence inside the step)
    first = lambda pat, after=t0: next(s for s, e, n, q in step if pat in n and s >= after)  # noqa: E731
    last = lambda pat: max(e for s, e, n, q in step if pat in n)  # noqa: E731
    m_embed_f = first("embed_fwd")
    m_embed_b = first("embed_bwd")
    m_attn_b = first("attn_dq_dma")
    end_adam = step[-1][1]
    phases = [("optimizer + trunk forward", t0, m_embed_f), ("encoder forward + head", m_embed_f, m_attn_b),
              ("encoder backward", m_attn_b, m_embed_b), ("embed + trunk backward + optimizer", m_embed_b, t1)]
    main_q = defaultdict(int)
    for s, e, n, q in step:
        main_q[q] += e - s
    mq = max(main_q, key=main_q.get)
    print(f"step {1e-6 * (t1 - t0):.2f} ms, {len(step)} dispatches; streams (busy ms): "
          + ", ".join(f"{q}: {1e-6 * v:.1f}" for q, v in sorted(main_q.items(), key=lambda kv: -kv[1])))
    for name, a, b in phases:
        iv = [(max(s, a), min(e, b)) for s, e, n, q in step if e > a and s < b]
        busy = union(iv)
        mine = union([x for x, (s, e, n, q) in zip(iv, [y for y in step if y[1] > a and y[0] < b]) if q == mq])
        # time with >= 2 kernels in flight
        ev = sorted([(s, 1) for s, e in iv] + [(e, -1) for s, e in iv])
        depth, last_t, multi = 0, None, 0
        for t, d in ev:
            if depth >= 2:
                multi += t - last_t
            depth += d
            last_t = t
        n = sum(1 for s, e, nm, q in step if a <= s < b)
        print(f"  {name:36s} wall {1e-6 * (b - a):7.2f} ms  busy {1e-6 * busy:7.2f}  idle {1e-6 * (b - a - busy):6.2f}"
              f"  overlapped {1e-6 * multi:6.2f}  main-stream busy {1e-6 * mine:7.2f}  dispatches {n}")


if __name__ == "__main__":
    main()
