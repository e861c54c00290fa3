"""Per-step decode kernel time of a VECTOR var / nested config from a rocprofv3
--stats summary: each decode kernel's average duration x its launches per
step (calls / K1's calls). python scripts/decode_sum.py profiles/r05/c3_kernel_stats.csv"""
import csv
import sys

DEC = ("vec_hdr_sample", "vec_hdr_kernel", "vec_tile_spec", "vec_tile_pick", "vec_tile_repair",
       "vec_tile_chain", "tscan_reduce", "tscan_apply", "vec_tile_emit", "vec_big_copy",
       "vec_tile_finish")
rows = list(csv.DictReader(open(sys.argv[1])))
k1 = [r for r in rows if "vec_tile_spec" in r["Name"]]
if not k1:
    sys.exit("no tile decode in this profile")
steps = int(k1[0]["Calls"])
tot = 0.0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].split("(")[0].replace("void ", "").replace("spk::", "")
    if not name.split("<")[0] in DEC:
        continue
    per = float(r["TotalDurationNs"]) / steps / 1e6
    tot += per
    print(f"{name:32s} {int(r['Calls']) / steps:5.2f}/step {float(r['AverageNs']) / 1e3:9.1f} us "
          f"{per:8.4f} ms/step")
print(f"decode kernel sum {tot:.4f} ms/step ({steps} steps)")
