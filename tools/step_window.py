"""Print one steady-state step of a rocprofv3 kernel trace: every dispatch between two
consecutive launches of the key kernel (default k_ex_chain; k_dt_part for the parallel
extrapolation mode), with queue, start/end (us, relative to the first key launch's end) and
duration.  usage: python tools/step_window.py TRACE.csv [STEP_INDEX [KEY]]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 30
key = sys.argv[3] if len(sys.argv) > 3 else 'k_ex_chain'
ch = [i for i, r in enumerate(rows) if r['Kernel_Name'] == key]
i0, i1 = ch[k], ch[k + 1]
t0 = int(rows[i0]['End_Timestamp'])
busy = {}
for r in rows[i0:i1 + 1]:
    s = int(r['Start_Timestamp']) - t0
    e = int(r['End_Timestamp']) - t0
    q = r['Queue_Id']
    busy[q] = busy.get(q, 0) + (e - s)
    print(f"{q:>2} {s / 1000:9.1f} {e / 1000:9.1f} {(e - s) / 1000:8.1f}  "
          f"{r['Kernel_Name'][:60]} g={r['Grid_Size_X']}")
per = int(rows[i1]['Start_Timestamp']) - int(rows[i0]['Start_Timestamp'])
print(f"period {per / 1000:.1f} us; busy per queue (us):",
      {q: round(b / 1000, 1) for q, b in busy.items()})
