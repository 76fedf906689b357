"""Summarise rocprofv3 --pmc passes (tools/pmc_fir.sh) per kernel:
effective clock, MFMA/VALU/LDS activity, LDS conflicts, and HBM traffic per launch with the
gfx950 correction (MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half of a wide coalesced
read, so it is doubled; WRITE_SIZE is exact for 16-B stores), calibrated against nsh_copy
whose traffic is known (16 B per sample). Writes a JSON summary."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def kernel_key(name):
    """'k_fir_mfma8<5>' from a demangled or an Itanium-mangled kernel name (rocprofv3 reports
    either, depending on the kernel's linkage), 'k_copy_v4' for the calibration copy."""
    m = re.search(r"(k_fir_\w+<[^>(]*>|k_copy_v4)", name)
    if m:
        return m.group(1).replace(" ", "")
    m = re.search(r"(k_chan1024|k_map_c_v4|k_fft1024)", name)  # the stream / FFT kernels, by base name
    if m:
        return m.group(1)
    m = re.search(r"\d(k_fir_[a-z0-9_]+?)I((?:L[ib]-?\d+E)+)E", name)
    if m:
        return "%s<%s>" % (m.group(1), ",".join(re.findall(r"L[ib](-?\d+)E", m.group(2))))
    return None


def main(root, n_samples, out_json):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in sorted(glob.glob(os.path.join(root, "p*"))):
        if not os.path.isdir(p):
            continue
        for r in load(p):
            k = r["Kernel_Name"]
            # key: the kernel template name, as nsh_fir_plan_kernel() reports it ("k_fir_mfma9<5>")
            short = kernel_key(k)
            if short is None:
                continue
            acc[short][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(short, r["Counter_Name"])].add(r["Dispatch_Id"])
    summ = {}
    for k, c in acc.items():
        nd = {cn: len(disp[(k, cn)]) for cn in c}
        per = {cn: v / max(nd[cn], 1) for cn, v in c.items()}  # per launch
        s = {"per_launch": per}
        if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
            rd = 2 * per["FETCH_SIZE"] * 1024  # KB -> B, x2 gfx950 wide-read correction
            wr = per["WRITE_SIZE"] * 1024
            s["hbm_read_bytes"] = rd
            s["hbm_write_bytes"] = wr
            s["hbm_bytes_per_sample"] = (rd + wr) / n_samples
        if "SQ_VALU_MFMA_BUSY_CYCLES" in per and "GRBM_GUI_ACTIVE" in per:
            s["mfma_busy_frac"] = per["SQ_VALU_MFMA_BUSY_CYCLES"] / (per["GRBM_GUI_ACTIVE"] / 8 * 256 * 4) if per["GRBM_GUI_ACTIVE"] else None
        if "SQ_WAVE_CYCLES" in per:
            w = per["SQ_WAVE_CYCLES"]
            s["wait_any_frac"] = per.get("SQ_WAIT_ANY", 0) / w if w else None
            s["wait_inst_frac"] = per.get("SQ_WAIT_INST_ANY", 0) / w if w else None
            s["active_frac"] = per.get("SQ_ACTIVE_INST_ANY", 0) / w if w else None
        summ[k] = s
    with open(out_json, "w") as f:
        json.dump(summ, f, indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
