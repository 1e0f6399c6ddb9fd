"""Per-kernel register / LDS / occupancy summary from hipcc -Rpass-analysis=kernel-resource-usage output."""
import re
import sys

for path in sys.argv[1:]:
    cur = None
    rows = []
    for line in open(path, errors="replace"):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key in ("VGPRs", "AGPRs", "SGPRs", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]",
                    "ScratchSize \\[bytes/lane\\]"):
            m = re.search(key + r": (\d+)", line)
            if m:
                cur[key.split(" ")[0].replace("\\", "")] = int(m.group(1))
    print("==", path)
    for r in rows:
        n = r["name"]
        m = re.search(r"fused_kernelILj(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELj(\d+)ELb(\d)", n)
        tag = f"fused GM={m.group(1)} K={m.group(2)} MB={m.group(3)} FILT={m.group(4)} WPE={m.group(6)} SEG={m.group(7)} MOVE={m.group(9)}" if m else n[:90]
        print(f"  {tag:70s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} sgpr={r.get('SGPRs')} occ={r.get('Occupancy')} lds={r.get('LDS')} scratch={r.get('ScratchSize')}")
