"""Compare the device ISA of two `hipcc --cuda-device-only -S` outputs kernel by kernel.

    python3 tools/isa_diff.py a.s b.s

Local labels are normalised, so a pure source move (a split into headers, reordered declarations)
prints "identical".  Used to check that refactors of csrc/ leave every kernel's code unchanged."""
import re
import sys


def kernels(path):
    text = open(path).read()
    out = {}
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end\d+:", text, re.S | re.M):
        body = re.sub(r"\.LBB\d+_\d+", "L", m.group(2))
        body = re.sub(r"\.Ltmp\d+", "T", body)
        body = re.sub(r"\.Lfunc_end\d+", "E", body)
        out[m.group(1)] = body
    # per-kernel resource metadata (.vgpr_count etc.) is in the amdhsa blocks
    for m in re.finditer(r"^\s*\.amdhsa_kernel (_Z\w+)\n(.*?)^\s*\.end_amdhsa_kernel", text, re.S | re.M):
        out[m.group(1)] += m.group(2)
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    only = sorted(set(a) ^ set(b))
    diff = sorted(k for k in a if k in b and a[k] != b[k])
    print(f"{len(a)} / {len(b)} kernels; only in one: {len(only)}; differing: {len(diff)}")
    for k in only + diff:
        print("  ", k)
    if not only and not diff:
        print("identical")
    return 1 if only or diff else 0


if __name__ == "__main__":
    sys.exit(main())
