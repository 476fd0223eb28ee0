"""Average PMC counters per kernel (per dispatch) from rocprofv3 counter CSVs."""
import csv, re, sys, collections

def short(name):
    m = re.match(r"(?:void )?(?:gnpde::)?([\w:]+)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]

acc = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        k = short(row["Kernel_Name"])
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        meta[k] = (row["Grid_Size"], row["VGPR_Count"], row["Accum_VGPR_Count"], row["LDS_Block_Size"])
for k in sorted(acc):
    d = {c: sum(v) / len(v) for c, v in acc[k].items()}
    print(f"== {k}  grid/vgpr/agpr/lds={meta[k]}")
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
    if "SQ_WAVE_CYCLES" in d and "SQ_WAVES" in d:
        print(f"   cycles/wave={d['SQ_WAVE_CYCLES']/d['SQ_WAVES']:.0f}  wait_any/wave_cyc={d.get('SQ_WAIT_ANY',0)/d['SQ_WAVE_CYCLES']:.2f}"
              f"  active_inst/wave_cyc={d.get('SQ_ACTIVE_INST_ANY',0)/d['SQ_WAVE_CYCLES']:.2f}")
