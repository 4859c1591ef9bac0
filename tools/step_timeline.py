"""One step of a rocprofv3 kernel trace laid out in time (for critical-path work).
    python tools/step_timeline.py <kernel_trace.csv> [step index]
Steps are delimited by the k_ex_chain launches; times are µs from the step's first kernel."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else -2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
chains = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_ex_chain"]
a, b = chains[k - 1] + 1, chains[k] + 1
# the step: from after the previous chain's last main-stream kernel to the chain after next
seg = rows[a:chains[k + 1] if k + 1 < len(chains) else len(rows)] if False else rows[a:b]
t0 = int(seg[0]["Start_Timestamp"])
for r in rows[a:] if False else rows[chains[k - 1] + 1:chains[k] + 1] + rows[chains[k] + 1:(chains[k + 1] if k + 1 < len(chains) else len(rows))]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r["Queue_Id"]:>2} {r["Kernel_Name"][:40]:40s} '
          f'grid {r["Grid_Size_X"]}x{r["Grid_Size_Y"]}')
