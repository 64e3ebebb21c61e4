#!/usr/bin/env python3
"""Per-kernel derived metrics from the passes of tools/pmc_eh.sh (serial solver run).

python tools/pmc_report.py gpurun_out/TAG [> profiles/xxx.md]

Counters of each kernel are averaged over its dispatches (every pass runs the same dispatch
sequence); durations come from each pass's kernel trace. Derived columns:
  VALU/wave, LDS/wave, VMEM/wave : instructions issued per wave (SQ_INSTS_* / SQ_WAVES)
  VALU busy %  : 100 * 4 * SQ_ACTIVE_INST_VALU / SIMDs / (GRBM_GUI_ACTIVE / 8): the SQ_ACTIVE_*
                 counters count quad-cycles summed over the chip, GRBM_GUI_ACTIVE is summed over
                 the 8 XCDs (MI355X_MICROARCH.md, PMC notes); rocprof's gfx94x VALUBusy formula
  LDS busy %   : the same normalisation of SQ_LDS_IDX_ACTIVE
  bank conf %  : 100 * SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  waves/CU     : mean resident waves per CU, 4 * SQ_WAVE_CYCLES (quad-cycles) over SQ_BUSY_CYCLES
                 per SQ (32 SQs)
Kernels launched at several sizes (the ECDSA bench sweeps batch sizes) get one row per grid size.
  rd GB, wr GB : FETCH_SIZE x 2 (gfx950 tallies 128-B reads at 64 B, MI355X_MICROARCH.md) and
                 WRITE_SIZE, per dispatch; TB/s over the dispatch's duration
"""
import collections
import csv
import glob
import re
import statistics
import sys

CUS = 256
SIMDS = 4 * CUS


def kname(name):
    m = re.search(r"eh_round<[^>]*>, (\d+), (?:false|true)>", name)
    if m:
        return "eh_round<%s>" % m.group(1)
    for k in ("eh_gen_reg", "eh_gen", "eh_expand", "eh_verify", "ecdsa_verify_kernel", "ecdsa_verify10h_kernel",
              "ecdsa_verify10_kernel", "ecdsa_fused_kernel", "ecdsa_prep_kernel"):
        if k in name:
            return k
    return re.sub(r"\(.*", "", name)[:40]


def main():
    d = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> values
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/*/*_counter_collection.csv")):
        rows = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k.startswith("ecdsa"):
                k += " n=%d" % (int(r.get("Grid_Size", 0) or 0))
            key = (r["Dispatch_Id"], k)
            rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[key]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for (_, k), cs in rows.items():
            for c, v in cs.items():
                if c == "_ns":
                    dur[k].append(v)
                else:
                    per[k][c].append(v)
    kernels = [k for k in per if k.startswith("eh_") or k.startswith("ecdsa")]
    kernels.sort(key=lambda k: (k.startswith("eh_round") and int(re.sub(r"\D", "", k)) or 0, k))

    def m(k, c):
        v = per[k].get(c)
        return statistics.mean(v) if v else float("nan")

    print("| kernel | µs | waves | VALU/wave | LDS/wave | SALU/wave | VMEM rd/wr per wave | VALU busy % | "
          "LDS busy % | bank conf % | waves/CU | rd GB | wr GB | TB/s |")
    print("|---" * 14 + "|")
    for k in kernels:
        us = statistics.median(dur[k]) / 1e3 if dur[k] else float("nan")
        w = m(k, "SQ_WAVES")
        gui = m(k, "GRBM_GUI_ACTIVE")
        rd = 2 * m(k, "FETCH_SIZE") * 1024 / 1e9
        wr = m(k, "WRITE_SIZE") * 1024 / 1e9
        tbs = (rd + wr) / (us * 1e-6) / 1e3 if us == us else float("nan")
        wpc = 4 * m(k, "SQ_WAVE_CYCLES") / max(m(k, "SQ_BUSY_CYCLES"), 1) / (CUS / 32)
        busy = lambda c: 100 * 4 * m(k, c) / SIMDS / (gui / 8)
        print(f"| {k} | {us:.0f} | {w:.0f} | {m(k, 'SQ_INSTS_VALU') / w:.0f} | {m(k, 'SQ_INSTS_LDS') / w:.0f} | "
              f"{m(k, 'SQ_INSTS_SALU') / w:.0f} | {m(k, 'SQ_INSTS_VMEM_RD') / w:.1f}/{m(k, 'SQ_INSTS_VMEM_WR') / w:.1f} | "
              f"{busy('SQ_ACTIVE_INST_VALU'):.0f} | {busy('SQ_LDS_IDX_ACTIVE'):.0f} | "
              f"{100 * m(k, 'SQ_LDS_BANK_CONFLICT') / max(m(k, 'SQ_LDS_IDX_ACTIVE'), 1):.0f} | {wpc:.1f} | "
              f"{rd:.2f} | {wr:.2f} | {tbs:.2f} |")


if __name__ == "__main__":
    main()
