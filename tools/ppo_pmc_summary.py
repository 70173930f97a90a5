"""Per-kernel summary of the PPO minibatch passes (tools/profile_round.sh step 3): trace
duration, HBM traffic (FETCH_SIZE doubled for the trunk kernels' 16-B/lane streaming reads,
MI355X_MICROARCH.md HBM note; WRITE_SIZE as reported), MFMA busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)) and, for the 96->96
trunk layers, achieved TFLOP/s on the algorithmic 2*N*P*96*96*9 flops of one launch."""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def label(name):
    """'k_bwd_data<bf16, 2, true, 13, true>' from a rocprofv3 kernel name: demangled
    ('(anonymous namespace)::k_bwd_data<2, true, ...>(...)') or, for the element-type
    templates rocprofv3 leaves mangled, '_ZN12_GLOBAL__N_110k_bwd_dataIDF16b...'."""
    if name.startswith("_ZN12_GLOBAL__N_1"):
        rest = name[len("_ZN12_GLOBAL__N_1"):]
        m = re.match(r"(\d+)", rest)
        n = int(m.group(1))
        base, rest = rest[len(m.group(1)):len(m.group(1)) + n], rest[len(m.group(1)) + n:]
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
    return re.match(r"\w+(<[^()]*>)?", short).group(0)


def layer96(lab):
    """the 96 -> 96 layers: forward / wgrad instantiated for 96 input channels (k_wgrad_c96 always), k_bwd_data's
    data-gradient variant (template argument DGRAD = true; the stem's has no dgrad)"""
    m = re.match(r"(\w+)<(.*)>$", lab)
    if not m:
        return False
    args = [a.strip() for a in m.group(2).split(",") if a.strip() not in ("bf16", "f16")]
    if m.group(1) in ("k_conv_gn_fwd", "k_wgrad"):
        return args[0] == "96"
    if m.group(1) == "k_wgrad_c96":  # 96 channels only
        return True
    return m.group(1) == "k_bwd_data" and args[1] == "true"

ap = argparse.ArgumentParser()
ap.add_argument("--fetch", required=True)
ap.add_argument("--write", required=True)
ap.add_argument("--mfma", required=True)
ap.add_argument("--trace", required=True)
ap.add_argument("--samples", type=int, default=32768)
ap.add_argument("--pixels", type=int, default=256)
ap.add_argument("--trunk-layers", type=int, default=10, help="96->96 layers one k_trunk_fwd / k_trunk_bwd launch runs")
ap.add_argument("--out", required=True)
a = ap.parse_args()


def counters(d, name):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(float)
        kern = {}
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != name:
                continue
            key = r.get("Dispatch_Id", r.get("Correlation_Id"))
            acc[key] += float(r["Counter_Value"])
            kern[key] = label(r["Kernel_Name"])
        for k, v in acc.items():
            per[kern[k]].append(v)
    return {k: sum(v) / len(v) for k, v in per.items()}


dur = defaultdict(list)
for f in glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[label(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
fe, wr = counters(a.fetch, "FETCH_SIZE"), counters(a.write, "WRITE_SIZE")
mb, gui = counters(a.mfma, "SQ_VALU_MFMA_BUSY_CYCLES"), counters(a.mfma, "GRBM_GUI_ACTIVE")
flops96 = 2.0 * a.samples * a.pixels * 96 * 96 * 9
rows = {}
for k, ds in dur.items():
    if not any(t in k for t in ("k_conv_gn_fwd", "k_bwd_data", "k_wgrad", "k_heads", "k_reduce", "k_trunk")):
        continue
    us = sum(ds) / len(ds)
    wide = any(t in k for t in ("k_conv_gn_fwd", "k_bwd_data", "k_wgrad", "k_heads", "k_trunk"))
    fb = fe.get(k, 0.0) * 1024 * (2 if wide else 1)
    wb = wr.get(k, 0.0) * 1024
    rec = {"launches": len(ds), "mean_us": us, "fetch_bytes": fb, "write_bytes": wb,
           "traffic_bytes": fb + wb, "hbm_GBps": (fb + wb) / (us * 1e-6) / 1e9 if us > 0 else None,
           "fetch_doubled": wide}
    if k in mb and gui.get(k):
        rec["mfma_busy_frac"] = mb[k] / (gui[k] / 8.0 * 1024.0)
        # GRBM_GUI_ACTIVE counts shader-clock cycles per XCD: over the traced duration, the kernel's
        # mean engine clock (MI355X peak 2.4 GHz; the MFMA peak scales with it)
        # (short kernels excluded: GRBM_GUI_ACTIVE also counts the dispatch's ramp and drain)
        if us >= 200.0:
            rec["sclk_GHz"] = gui[k] / 8.0 / (us * 1e3)
    nl = a.trunk_layers if k.startswith("k_trunk") else (1 if layer96(k) else 0)
    if nl:  # a k_trunk_* launch runs every 96->96 layer of the stack (the backward's stem has no dgrad)
        rec["layers96"] = nl
        rec["algo_tflop"] = nl * flops96 / 1e12
        rec["achieved_TFLOPs"] = nl * flops96 / (us * 1e-6) / 1e12
        rec["mfma_frac_of_2500"] = rec["achieved_TFLOPs"] / 2500.0
    rows[k] = rec
json.dump({"samples": a.samples, "kernels": rows}, open(a.out, "w"), indent=1)
for k, r in sorted(rows.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["launches"]):
    print(f"{r['mean_us']:9.1f} us x{r['launches']:3d} traffic {r['traffic_bytes'] / 1e9:6.2f} GB "
          f"mfma_busy {r.get('mfma_busy_frac', float('nan')):.3f} sclk {r.get('sclk_GHz', float('nan')):.2f} GHz {k[:90]}")
