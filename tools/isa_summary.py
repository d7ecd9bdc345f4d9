"""Per-kernel summary of a gfx950 device assembly file (hipcc --cuda-device-only -S):
VGPRs, occupancy, and the order of the memory instructions and waits, to check that a
streaming loop keeps its loads in flight.

  python tools/isa_summary.py FILE.s SUBSTRING [SUBSTRING ...] [--ops N]
"""
import re
import sys


def kernels(text):
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\S+):", text, re.M)]
    for i, (pos, name) in enumerate(starts):
        end = starts[i + 1][0] if i + 1 < len(starts) else len(text)
        yield name, text[pos:end]


def main(argv):
    ops = 80
    if "--ops" in argv:
        i = argv.index("--ops")
        ops = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    path, subs = argv[0], argv[1:]
    text = open(path).read()
    for name, body in kernels(text):
        if not all(s in name for s in subs):
            continue
        vg = re.search(r"NumVgprs:\s*(\d+)", body)
        oc = re.search(r"Occupancy:\s*(\d+)", body)
        sc = re.search(r"ScratchSize:\s*(\d+)", body)
        seq = []
        for line in body.split("\n"):
            t = line.strip().split()
            if not t:
                continue
            op = t[0]
            if op.startswith(("global_load", "global_store", "buffer_load", "s_load", "ds_read", "ds_write")) or \
                    op in ("s_waitcnt", "s_barrier", "s_cbranch_vccnz", "s_cbranch_scc1", "s_cbranch_scc0",
                           "s_cbranch_execz", "s_branch"):
                seq.append(op + (" " + t[1] if op == "s_waitcnt" else ""))
        print(f"{name[:110]}\n  vgpr={vg and vg.group(1)} occupancy={oc and oc.group(1)} "
              f"scratch={sc and sc.group(1)} global_loads={sum(s.startswith('global_load') for s in seq)}")
        print("  " + " | ".join(seq[:ops]))


if __name__ == "__main__":
    main(sys.argv[1:])
