"""Per-function resource summary of a hipcc --save-temps gfx950 assembly file: instruction count,
VGPR/AGPR use, scratch bytes, scratch loads/stores, calls.

    python tools/isa_stats.py /tmp/bn256-hip-amdgcn-amd-amdhsa-gfx950.s
"""
import re
import sys


def main(path):
    s = open(path).read()
    for m in re.finditer(r"^(\S+):\s+; @(\S+)\n", s, re.M):
        name = m.group(1)
        end = s.find("; -- End function", m.end())
        body = s[m.end():end]
        tail = s[end:end + 4000]
        lines = [l for l in body.split("\n") if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]

        def g(k):
            mm = re.search(r"; " + k + r":\s*(\d+)", tail)
            return int(mm.group(1)) if mm else -1
        print(f"{name[:58]:58s} inst={len(lines):6d} vgpr={g('NumVgprs'):3d} agpr={g('NumAgprs'):3d} "
              f"scratch={g('ScratchSize'):6d} st={sum('scratch_store' in l for l in lines):5d} "
              f"ld={sum('scratch_load' in l for l in lines):5d} acc={sum('accvgpr' in l for l in lines):5d} "
              f"calls={sum('s_swappc' in l for l in lines):4d}")


if __name__ == "__main__":
    main(sys.argv[1])
