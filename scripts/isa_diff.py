"""Compare the gfx950 ISA of kernels between two builds of libgenpose_hip.so (tuning aid, not a test).

    python scripts/isa_diff.py OLD.so NEW.so [regex]     # default regex: every kernel

Prints, per kernel matching the regex, whether the instruction streams (addresses and branch offsets
stripped) are identical, else the instruction counts and the first differing lines.
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_cpu_host import _gfx950_code_objects  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def kernels(so):
    out = {}
    for co in _gfx950_code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name], capture_output=True, text=True,
                                 check=True).stdout
        for fn, body in re.findall(r"^[0-9a-f]+ <(\w+)>:\n(.*?)(?=^[0-9a-f]+ <|\Z)", dis, re.M | re.S):
            ins = []
            for line in body.split("\n"):
                code = re.sub(r"<[^>]*>", "", line.split("//")[0]).strip()
                if code:
                    ins.append(code)
            out[fn] = ins
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    pat = re.compile(sys.argv[3] if len(sys.argv) > 3 else ".")
    for fn in sorted(set(a) | set(b)):
        if not pat.search(fn):
            continue
        if fn not in a or fn not in b:
            print(f"{'only new' if fn not in a else 'only old'}: {fn}")
            continue
        if a[fn] == b[fn]:
            print(f"same ({len(a[fn])}): {fn}")
            continue
        i = next(k for k, (x, y) in enumerate(zip(a[fn] + [""], b[fn] + [""])) if x != y)
        print(f"DIFF ({len(a[fn])} -> {len(b[fn])}): {fn}\n   old[{i}]: {a[fn][i] if i < len(a[fn]) else ''}\n"
              f"   new[{i}]: {b[fn][i] if i < len(b[fn]) else ''}")


if __name__ == "__main__":
    main()
