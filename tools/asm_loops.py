"""List the loops of one kernel in a hipcc -save-temps .s with their instruction mix."""
import re
import sys
from collections import Counter

path, name = sys.argv[1], sys.argv[2]
s = open(path).read()
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
body = s[i:j].split("\n")
labels = {l.split(";")[0].strip()[:-1]: k for k, l in enumerate(body) if l.startswith(".LBB") and l.split(";")[0].strip().endswith(":")}
for k, l in enumerate(body):
    t = l.strip().split()
    if t and t[0].startswith("s_cbranch") or (t and t[0] == "s_branch"):
        if len(t) > 1 and t[1] in labels and labels[t[1]] < k:
            seg = [x.strip().split()[0] for x in body[labels[t[1]]:k + 1] if x.strip() and not x.strip().startswith(";") and not x.strip().startswith(".")]
            c = Counter(seg)
            f64 = sum(v for op, v in c.items() if op.startswith("v_") and "f64" in op)
            print(f"loop {t[1]} len {k - labels[t[1]]} f64 {f64} scratch {sum(v for op, v in c.items() if 'scratch' in op)} "
                  f"ds {sum(v for op, v in c.items() if op.startswith('ds_'))} ldexp {c.get('v_ldexp_f64', 0)} readlane {c.get('v_readlane_b32', 0)}")
