"""Audit of device assembly (hipcc --cuda-device-only -S): for every kernel
whose name matches a pattern, the loops (LLVM 'Loop Header' labels) and the
vmcnt waits / global loads / MFMAs inside each loop body.  A vmcnt(0) inside a
software-pipelined loop drains every load in flight (no latency hiding).

    python tools/loop_waitcnt.py conv.s [name-substring ...]"""
import re
import sys


def kernels(lines):
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l)]
    for k, (i, name) in enumerate(starts):
        end = starts[k + 1][0] if k + 1 < len(starts) else len(lines)
        yield name, lines[i:end]


def main():
    lines = open(sys.argv[1]).read().split("\n")
    pats = sys.argv[2:]
    for name, body in kernels(lines):
        if pats and not any(p in name for p in pats):
            continue
        heads = [i for i, l in enumerate(body) if "Loop Header" in l]
        out = []
        for h in heads:
            lab = body[h].split(":")[0]
            # loop extent: last backward branch to this label
            ends = [i for i, l in enumerate(body) if i > h and re.search(r"s_c?branch\w*\s+%s\b" % re.escape(lab), l)]
            if not ends:
                continue
            e = max(ends)
            seg = body[h:e + 1]
            vm = [re.search(r"vmcnt\((\d+)\)", l).group(1) for l in seg if "vmcnt(" in l]
            nl = sum(1 for l in seg if re.search(r"global_load|buffer_load", l))
            nm = sum(1 for l in seg if "v_mfma" in l)
            if nl == 0 and nm == 0:
                continue
            out.append("  loop %s: %d lines, %d loads, %d mfma, vmcnt waits %s" % (lab, len(seg), nl, nm, ",".join(vm)))
        if out:
            print(name)
            print("\n".join(out))


if __name__ == "__main__":
    main()
