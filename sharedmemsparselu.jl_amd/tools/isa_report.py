"""Dev helper: per-kernel memory-instruction mix of a gfx950 assembly dump (hipcc -S)."""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\S+):', s, re.M):
    name = m.group(1)
    i = m.end()
    j = s.find('.Lfunc_end', i)
    b = s[i:j]
    vg = re.search(r'; NumVgprs: (\d+)', s[j:j + 4000])
    ag = re.search(r'; NumAgprs: (\d+)', s[j:j + 4000])
    sc = re.search(r'; ScratchSize: (\d+)', s[j:j + 4000])
    print(f"{name[:60]:60s} flat {b.count('flat_load'):4d}/{b.count('flat_store'):4d} "
          f"global {b.count('global_load'):4d}/{b.count('global_store'):4d} "
          f"vgpr {vg and vg.group(1)} agpr {ag and ag.group(1)} scratch {sc and sc.group(1)}")
