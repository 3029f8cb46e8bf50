"""Summarise kernels in a hipcc `-save-temps` gfx950 assembly file: register budget,
scratch use and the s_waitcnt mix (a `vmcnt(0)` inside a streaming loop means the
prefetch pipeline was drained).

    python tools/isa_report.py <file.s> [substring-of-mangled-name ...]
"""
import re
import sys
from collections import Counter


def report(path, pats):
    s = open(path).read()
    names = re.findall(r"^(_Z\S+):", s, re.M)
    for name in names:
        if pats and not any(p in name for p in pats):
            continue
        i = s.find(name + ":")
        j = s.find(".Lfunc_end", i)
        body = s[i:j]
        k = s.find(".amdhsa_kernel " + name)
        seg = s[k:k + 3000]
        meta = {}
        for key in (".amdhsa_next_free_vgpr", ".amdhsa_accum_offset", ".amdhsa_next_free_sgpr",
                    ".amdhsa_private_segment_fixed_size", ".amdhsa_group_segment_fixed_size"):
            m = re.search(re.escape(key) + r"\s+(\d+)", seg)
            meta[key.split("_", 1)[1]] = int(m.group(1)) if m else None
        waits = Counter(re.findall(r"s_waitcnt[^\n;]*", body))
        glds = body.count("global_load_lds")
        gl = len(re.findall(r"global_load_dword", body)) - glds
        print(name[:90])
        print("   ", meta)
        print("    glds", glds, "global_load", gl, "scratch", body.count("scratch_"),
              "ds_read", body.count("ds_read"), "waits:", dict(waits.most_common(8)))


if __name__ == "__main__":
    report(sys.argv[1], sys.argv[2:])
