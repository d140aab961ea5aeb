"""GPU idle time of a rocprofv3 kernel trace (--kernel-trace --output-format csv):
    python tools/trace_gaps.py <kernel_trace.csv> [t_from_s t_to_s]
Merges every kernel's [start, end] interval (all queues) and reports, over the traced span (or the
given window, seconds from the first kernel), busy time, idle time, the largest idle gaps and the
kernels that precede them (what the GPU waited on the host after)."""
import csv
import re
import sys


def short(n):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.split(r"[<(]", n)[0][:48]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t0 = iv[0][0]
    lo = t0 + int(float(sys.argv[2]) * 1e9) if len(sys.argv) > 3 else t0
    hi = t0 + int(float(sys.argv[3]) * 1e9) if len(sys.argv) > 3 else max(e for _, e, _ in iv)
    busy, gaps, cur_s, cur_e, prev = 0, [], None, None, None
    for s, e, n in iv:
        if e < lo or s > hi:
            continue
        s, e = max(s, lo), min(e, hi)
        if cur_e is None:
            cur_s, cur_e, prev = s, e, n
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n, cur_e - t0))
            cur_s, cur_e, prev = s, e, n
        else:
            if e > cur_e:
                cur_e, prev = e, n
    busy += cur_e - cur_s
    span = hi - lo
    idle = span - busy
    print(f"span {span / 1e9:.2f} s  busy {busy / 1e9:.2f} s  idle {idle / 1e9:.2f} s "
          f"({100 * idle / span:.1f} %)  gaps {len(gaps)}")
    big = [g for g in gaps if g[0] > 1e5]
    print(f"gaps > 0.1 ms: {len(big)} totalling {sum(g[0] for g in big) / 1e9:.2f} s")
    by = {}
    for g, p, n, _ in gaps:
        k = short(p)
        by[k] = by.get(k, 0) + g
    hist = [0, 0, 0, 0, 0]
    for g, _, _, _ in gaps:
        hist[min(4, sum(g > t for t in (1e4, 1e5, 1e6, 1e7)))] += g
    print("idle by gap size  <10us %.2f s | 10-100us %.2f s | 0.1-1ms %.2f s | 1-10ms %.2f s | "
          ">10ms %.2f s" % tuple(h / 1e9 for h in hist))
    for k, v in sorted(by.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  idle after {k:60s} {v / 1e9:8.3f} s")
    for g, p, n, at in sorted(gaps, reverse=True)[:15]:
        print(f"  {g / 1e6:9.2f} ms at {at / 1e9:8.2f} s after {short(p)} -> {short(n)}")


if __name__ == "__main__":
    main()
