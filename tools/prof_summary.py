"""Turn one gpurun profiling session (tools/gpu_profile.sh TAG) into the committed
evidence under profiles/:

  profiles/<TAG>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (rocpd2summary)
  profiles/<TAG>_pmc.json           per-kernel FETCH_SIZE / WRITE_SIZE (separate --pmc passes)
  profiles/pmc_traffic_<wl>.json    HBM bytes per launch of the dominant kernels, read by bench.py

HBM traffic follows MI355X_MICROARCH.md (rocprofv3 section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of wide streaming reads,
so traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).

usage: python tools/prof_summary.py TAG WORKLOAD [KERNEL_SUBSTRINGS]   (tools/gpu_profile.sh layout)
"""
import csv
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(path, counter):
    out = {}
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        out.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    tag, wl = sys.argv[1], sys.argv[2]
    kern = sys.argv[3] if len(sys.argv) > 3 else "k_decode,k_fast_merge"
    src = os.path.join(ROOT, "gpurun_out", tag)
    prof = os.path.join(ROOT, "profiles", tag[:3])
    os.makedirs(prof, exist_ok=True)
    tag = f"{tag}_{wl}"
    kt = os.path.join(src, f"kt_{wl}")
    dbs = [os.path.join(dp, f) for dp, _, fs in os.walk(kt) for f in fs if f.endswith(".db")]
    stats = [os.path.join(dp, f) for dp, _, fs in os.walk(kt) for f in fs if f.endswith("kernel_stats.csv")]
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    elif dbs:
        tmp = tempfile.mkdtemp()
        subprocess.check_call(["/opt/rocm/bin/rocpd2summary", "-i", dbs[0], "-d", tmp, "--format", "csv"],
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        shutil.copy(os.path.join(tmp, "kernels_summary.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = pmc(os.path.join(src, f"pmc_fetch_{wl}", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, f"pmc_write_{wl}", "pmc_counter_collection.csv"), "WRITE_SIZE")
    res = {"tag": tag, "unit": "KiB per launch (mean over launches)", "fetch_size": fetch, "write_size": write}
    if fetch or write:
        with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
            json.dump(res, f, indent=1)
    # KERNEL_SUBSTRING may list several kernels ("k_decode,k_fast_merge"): the dominant
    # stage is then their sum per step, matching bench.py's combined kernel_ms.
    names = kern.split(",")
    fk = [next((k for k in fetch if n in k), None) for n in names]
    wk = [next((k for k in write if n in k), None) for n in names]
    if all(fk) and all(wk):
        fs = sum(fetch[k] for k in fk)
        ws = sum(write[k] for k in wk)
        t = (2 * fs + ws) * 1024
        with open(os.path.join(ROOT, "profiles", f"pmc_traffic_{wl}.json"), "w") as f:
            json.dump({"tag": tag, "workload": wl, "kernel": " + ".join(fk), "fetch_kib": fs, "write_kib": ws,
                       "traffic_bytes_per_launch": t,
                       "formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)"},
                      f, indent=1)
        print(f"{kern}: traffic {t / 1e6:.1f} MB per launch")
    for n in (f"bench_{wl}.log", "stamps.log", "pytest_gpu.log", "smoke.log"):
        p = os.path.join(src, n)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(prof, f"{tag}_{n}"))


if __name__ == "__main__":
    main()
