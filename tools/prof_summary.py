"""Turn one gpurun profiling session (tools/gpu_profile.sh TAG) into the committed
evidence under profiles/:

  profiles/<TAG>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (rocpd2summary)
  profiles/<TAG>_pmc.json           per-kernel FETCH_SIZE / WRITE_SIZE (separate --pmc passes)
  profiles/pmc_traffic.json         HBM bytes per launch of the dominant kernel, read by bench.py

HBM traffic follows MI355X_MICROARCH.md (rocprofv3 section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of wide streaming reads,
so traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).

usage: python tools/prof_summary.py TAG [KERNEL_SUBSTRING]
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
    tag = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "k_fast_merge"
    src = os.path.join(ROOT, "gpurun_out", tag)
    prof = os.path.join(ROOT, "profiles")
    dbs = [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(src, "kt")) for f in fs if f.endswith(".db")]
    stats = [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(src, "kt")) for f in fs
             if f.endswith("kernel_stats.csv")]
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    elif dbs:
        tmp = tempfile.mkdtemp()
        subprocess.check_call(["/opt/rocm/bin/rocpd2summary", "-i", dbs[0], "-d", tmp, "--format", "csv"],
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        shutil.copy(os.path.join(tmp, "kernels_summary.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = pmc(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    res = {"tag": tag, "unit": "KiB per launch (mean over launches)", "fetch_size": fetch, "write_size": write}
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(res, f, indent=1)
    fk = [k for k in fetch if kern in k]
    wk = [k for k in write if kern in k]
    if fk and wk:
        t = (2 * fetch[fk[0]] + write[wk[0]]) * 1024
        with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
            json.dump({"tag": tag, "kernel": fk[0], "fetch_kib": fetch[fk[0]], "write_kib": write[wk[0]],
                       "traffic_bytes_per_launch": t,
                       "formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)"},
                      f, indent=1)
        print(f"{kern}: traffic {t / 1e6:.1f} MB per launch")
    for n in ("bench.log", "stamps.log", "pytest_gpu.log"):
        p = os.path.join(src, n)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(prof, f"{tag}_{n}"))


if __name__ == "__main__":
    main()
