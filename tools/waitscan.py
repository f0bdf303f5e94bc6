#!/usr/bin/env python3
"""Per-kernel count of vector loads that are waited on (vmcnt(0)) within the
next few instructions -- the signature of a load whose latency is exposed
(e.g. a load inside a divergent branch)."""
import re, sys
s = open(sys.argv[1]).read()
labels = [(m.start(), m.group(1)) for m in re.finditer(r'^(_ZN7surfhip\w+):', s, re.M)]
for i, (pos, name) in enumerate(labels):
    end = labels[i + 1][0] if i + 1 < len(labels) else len(s)
    body = s[pos:end].split('s_endpgm')[0].split('\n')
    loads = [j for j, l in enumerate(body) if re.search(r'\b(global|buffer)_load', l)]
    exposed = sum(1 for j in loads if any('vmcnt(0)' in body[k] for k in range(j + 1, min(j + 4, len(body)))))
    waits = sum('s_waitcnt vmcnt' in l for l in body)
    print(f"{name[12:70]:58s} loads {len(loads):4d}  exposed {exposed:3d}  vmcnt waits {waits:3d}")
