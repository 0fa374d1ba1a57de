"""Per-kernel SGPR-spill traffic in a gfx950 assembly listing (hipcc -S
--cuda-device-only): v_writelane / v_readlane counts (how SGPR spills to
VGPR lanes are coded), VALU and SALU instruction counts, static.
usage: python tools/isa_spills.py FILE.s [NAME_REGEX]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
for m in re.finditer(r'^(_Z\S*?):\s*;\s*@', s, re.M):
    n = m.group(1)
    if pat and not pat.search(n):
        continue
    j = s.find('.Lfunc_end', m.end())
    body = s[m.end():j]
    print("%-70s writelane %4d readlane %4d valu %5d salu %5d" % (
        n[:70], body.count('v_writelane'), body.count('v_readlane'),
        len(re.findall(r'^\s+v_', body, re.M)), len(re.findall(r'^\s+s_', body, re.M))))
