"""Turn rocprofv3 --pmc counter_collection.csv files into per-launch HBM traffic per kernel.

Usage: python tools/pmc_traffic.py OUT.json FETCH_DIR WRITE_DIR
  FETCH_DIR: a `rocprofv3 --pmc FETCH_SIZE` pass, WRITE_DIR: a `rocprofv3 --pmc WRITE_SIZE` pass
  (separate passes: FETCH_SIZE needs 3 TCC counters, WRITE_SIZE 2, the TCC block holds 4).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KB. On gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read; other access widths
are uncalibrated. Both figures are therefore written per launch: `bytes_per_launch` = (FETCH_SIZE +
WRITE_SIZE) * 1024 (raw, no correction: the lower bound, and the value bench.py reports as `traffic`)
and `bytes_fetch_doubled` = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (the guide's correction, exact for
16-B/lane streaming reads, an upper bound for narrower ones).
Kernel names are mapped to the bench.py stage names below. The factorization ("chol_factor") is a
chain of launches (scatter, extend-add, panel steps, trailing updates): its traffic is the sum over
all of its dispatches divided by the number of factorizations (k_chol_scatter, which also initialises the front
vectors, runs once per factorization; k_vec_init counts where no level is pre-scattered).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

STAGES = {  # substring of the kernel name -> stage name used by bench.py (a stage's kernels each run once per
    # iteration: the stage's traffic per launch is the sum of its kernels' per-dispatch means)
    "k_schur_rows": "schur_rows",
    "k_schur_prep": "schur_dinv",
    "k_schur_diag": "schur_diag",
    "k_linearize": "linearize",
    "k_backsub": "backsub",
    "k_vertex_reduce": "vreduce",
    "k_cam_assemble": "vreduce",  # fused BA assembly (assembly.hip): the camera pass + landmark fix-ups
    "k_lm_fixup": "vreduce",
}


FACTOR = ("k_zero_ranges", "k_chol_scatter", "k_vec_init", "k_extend_add", "k_step", "k_syrk", "k_permute")


def _split_variant(name):
    """None for kernels without a Schur-split variant, else True / False (assembly.hip templates)."""
    if not any(k in name for k in ("k_linearize_fused", "k_cam_assemble", "k_lm_fixup")):
        return None
    return ", true>" in name or "<true>" in name


def read_counter(d, counter):
    per = defaultdict(list)
    fsum, nscat, nvec = 0.0, 0, 0
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == counter]
    # iteration 0 of the LM loop assembles without the Schur split (lambda unknown): when split dispatches are
    # present, the plain variants of the assembly kernels are left out of the per-launch figures
    has_split = any(_split_variant(r.get("Kernel_Name", "")) for r in rows)
    for r in rows:
        name = r.get("Kernel_Name", "")
        if has_split and _split_variant(name) is False:
            continue
        for sub in STAGES:
            if sub in name:
                per[sub].append(float(r["Counter_Value"]))
        if any("::" + k + "(" in name or "::" + k + "<" in name for k in FACTOR):
            fsum += float(r["Counter_Value"])
            nscat += "::k_chol_scatter(" in name
            nvec += "::k_vec_init(" in name
    st = defaultdict(list)
    for sub, vals in per.items():  # per stage: sum of its kernels' per-dispatch means, one entry per dispatch
        st[STAGES[sub]].append((sum(vals) / len(vals), len(vals)))
    out = {k: [sum(m for m, _ in v)] * max(n for _, n in v) for k, v in st.items()}
    nfac = nscat or nvec
    if nfac:
        out["chol_factor"] = [fsum / nfac] * nfac
    return out


def main():
    out, fdir, wdir = sys.argv[1:4]
    fetch = read_counter(fdir, "FETCH_SIZE")
    write = read_counter(wdir, "WRITE_SIZE")
    res = {}
    for stage in sorted(set(fetch) | set(write)):
        if not fetch.get(stage) or not write.get(stage):
            continue
        f = sum(fetch[stage]) / len(fetch[stage])
        w = sum(write[stage]) / len(write[stage])
        res[stage] = {
            "bytes_per_launch": (f + w) * 1024.0,
            "bytes_fetch_doubled": (2.0 * f + w) * 1024.0,
            "fetch_size_kb_raw": f,
            "write_size_kb": w,
            "launches": len(fetch[stage]),
            "correction": "bytes_per_launch: (FETCH_SIZE + WRITE_SIZE) * 1024, raw; bytes_fetch_doubled: "
                          "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 half-count of 16-B/lane streaming reads)",
        }
        if stage == "chol_factor":
            res[stage]["launches"] = "factorizations (sum over the factor's kernel chain)"
    res["_meta"] = {"config": os.environ.get("G2OHIP_TRAFFIC_CONFIG", "C4"),
                    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py, tools/pmc_traffic.py"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
