"""Wave-state and MFMA-busy fractions per trunk kernel variant from one rocprofv3 --pmc pass
(tools/ws_sq_pass.sh): parked = SQ_WAIT_ANY, issue-stalled = SQ_WAIT_INST_ANY, issuing =
SQ_ACTIVE_INST_ANY, each / SQ_WAVE_CYCLES; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), summed over each kernel's dispatches.
    python tools/ws_sq_summary.py --pmc DIR --out FILE.csv"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict



def label(name):
    """'k_conv_gn_fwd_ws3<f16, 96, 8, true, false>' from a rocprofv3 kernel name (mangled
    element-type templates, or demangled '(anonymous namespace)::k_...<...>(...)')."""
    if name.startswith("_ZN12_GLOBAL__N_1"):
        rest = name[len("_ZN12_GLOBAL__N_1"):]
        n = int(re.match(r"(\d+)", rest).group(1))
        d = len(str(n))
        base, rest = rest[d:d + n], rest[d + n:]
        args = []
        if rest.startswith("I"):
            i = 1
            while i < len(rest) and rest[i] != "E":
                if rest.startswith("DF16b", i):
                    args.append("bf16"); i += 5
                elif rest.startswith("DF16_", i):
                    args.append("f16"); i += 5
                elif rest.startswith("Lb", i):
                    args.append("true" if rest[i + 2] == "1" else "false"); i += 4
                elif rest.startswith("Li", i):
                    j = rest.index("E", i)
                    args.append(rest[i + 2:j]); i = j + 1
                else:
                    break
        return f"{base}<{', '.join(args)}>" if args else base
    short = name.split("(anonymous namespace)::", 1)[-1]
    m = re.match(r"\w+(<[^()]*>)?", short)
    return m.group(0) if m else short

ap = argparse.ArgumentParser()
ap.add_argument("--pmc", required=True)
ap.add_argument("--out", required=True)
a = ap.parse_args()
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(a.pmc, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = label(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id")))
rows = []
for k, c in sorted(acc.items()):
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    g = c.get("GRBM_GUI_ACTIVE", 0.0)
    if wc <= 0 or not k.startswith("k_"):
        continue
    rows.append(dict(kernel=k, dispatches=len(disp[k]), parked=c.get("SQ_WAIT_ANY", 0) / wc,
                     issue_stalled=c.get("SQ_WAIT_INST_ANY", 0) / wc, issuing=c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                     mfma_busy=(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (g / 8 * 1024)) if g > 0 else float("nan")))
with open(a.out, "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) if rows else ["kernel"])
    w.writeheader()
    for r in rows:
        w.writerow({k: (f"{v:.3f}" if isinstance(v, float) else v) for k, v in r.items()})
for r in rows:
    print(f"{r['kernel']:48s} x{r['dispatches']:3d} parked {r['parked']:.3f} issue-stalled {r['issue_stalled']:.3f} "
          f"issuing {r['issuing']:.3f} mfma busy {r['mfma_busy']:.3f}")
