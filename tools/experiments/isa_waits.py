"""Print the memory-wait skeleton of one kernel in a device .s file:
global loads, vmcnt waits, barriers, labels and branches (to check that
loads stay in flight where a kernel means them to).

usage: python tools/experiments/isa_waits.py file.s mangled_kernel_name_substring
"""
import re
import sys

src, want = sys.argv[1], sys.argv[2]
text = open(src).read()
start = next(m.start() for m in re.finditer(r"^([A-Za-z_.$][^\s:]*):", text, re.M) if want in m.group(1))
end = text.find(".Lfunc_end", start)
lines = text[start:end].split("\n")
print(f"{len(lines)} lines")
for n, line in enumerate(lines):
    if re.search(r"vmcnt|s_barrier|global_load|scratch_|^\.LBB|s_cbranch", line):
        print(n, line.strip())
