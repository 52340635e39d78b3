"""Per-step busy and idle time of a rocprofv3 kernel trace: a step starts at each launch of
the given kernel (config 5: the position-stage `k_all_humanoid<false>`, once per
mjd_inverseFD call). Steps whose span is far above the median (warm-up edges, host work
between the timed regions) are left out.

  python tools/trace_idle.py profiles/r05/head2/c5_kernel_trace.csv [first_kernel_prefix]
"""
import csv
import statistics
import sys


def main():
  path = sys.argv[1]
  first = sys.argv[2] if len(sys.argv) > 2 else "void k_all_humanoid<false>"
  rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
  idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(first)]
  steps = []
  for a, b in zip(idx[:-1], idx[1:]):
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b])
    steps.append(((t1 - t0) / 1e3, busy / 1e3))
  med = statistics.median(s for s, _ in steps)
  inner = [(s, b) for s, b in steps if s < 2 * med]
  span, busy = sum(s for s, _ in inner), sum(b for _, b in inner)
  print(f"{len(inner)} steps (of {len(steps)}): span {span / len(inner):.1f} us/step, "
        f"kernels {busy / len(inner):.1f} us/step, idle {100 * (span - busy) / span:.2f}%")


if __name__ == "__main__":
  main()
