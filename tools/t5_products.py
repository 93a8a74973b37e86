"""Per-product kernel times of the frozen T5 encoder from rocprofv3 kernel traces of
tools/t5_encoder_probe.py (tools/gpu_t5_variants.sh): the GEMM launches of each layer in order
(QKV, o-projection + residual, FF-in relu, FF-out + residual), median over layers and replays.
Usage: t5_products.py DIR [DIR ...]"""
import csv
import glob
import statistics
import sys

NAMES = ("qkv", "o_proj", "ff_in", "ff_out")
for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    g = [r for r in rows if "gemm" in r["Kernel_Name"]]
    per = {n: [] for n in NAMES}
    kern = {}
    for i, r in enumerate(g):
        n = NAMES[i % 4]
        per[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        kern[n] = r["Kernel_Name"].split("(")[0].replace("void (anonymous namespace)::", "")
    tot = sum(statistics.median(v) for v in per.values())
    print(f"{d}: " + "  ".join(f"{n} {statistics.median(per[n]):6.1f} us [{kern[n][:40]}]" for n in NAMES)
          + f"  sum {tot:.1f}")
