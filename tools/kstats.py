"""Per-kernel average durations from a rocprofv3 kernel_stats.csv (short names)."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in list(csv.reader(open(path)))[1:]:
        n = r[0].replace("tvm::(anonymous namespace)::", "").replace("void ", "")
        n = re.sub(r"rocprim::ROCPRIM_\w+::detail::", "rocprim::", n)
        n = re.split(r"\(", n)[0][:70]
        print(f"  {n:70s} {int(r[1]):5d} {float(r[3]) / 1e3:9.1f} us")
