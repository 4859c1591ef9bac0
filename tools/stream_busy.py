"""Per-queue busy time and idle gaps per step from a rocprofv3 kernel trace (which stream
binds the step).  Steps are delimited by the launches of a marker kernel (default k_mom_prep,
the first kernel of a step on the main stream).
    python tools/stream_busy.py <kernel_trace.csv> [marker] [first step] [last step]"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "k_mom_prep"
marks = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"] == marker]
a = int(sys.argv[3]) if len(sys.argv) > 3 else len(marks) // 2
b = int(sys.argv[4]) if len(sys.argv) > 4 else len(marks) - 2
t0, t1 = marks[a], marks[b]
n = b - a
busy, kern = defaultdict(float), defaultdict(lambda: defaultdict(float))
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    s, e = max(s, t0), min(e, t1)
    if e <= s:
        continue
    q = r["Queue_Id"]
    busy[q] += e - s
    kern[q][r["Kernel_Name"][:32]] += e - s
print(f"steps {a}..{b}: period {(t1 - t0) / n / 1e3:.1f} us")
for q in sorted(busy):
    print(f"queue {q}: busy {busy[q] / n / 1e3:8.1f} us/step")
    for k, v in sorted(kern[q].items(), key=lambda kv: -kv[1])[:14]:
        print(f"    {v / n / 1e3:8.1f}  {k}")
