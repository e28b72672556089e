import re,sys
def load(p):
    d=[]
    for line in open(p):
        m=re.match(r"\s+([0-9.]+) (.*)",line)
        if m and not line.strip().startswith("step"): d.append((float(m.group(1)),m.group(2)[:60]))
    return d
a=load(sys.argv[1]); others=[load(p) for p in sys.argv[2:]]
for i,(t,n) in enumerate(a):
    if "us  " in n: continue
    print(f"{t:7.2f} "+" ".join(f"{o[i][0]:7.2f}" if i<len(o) else "   -   " for o in others)+"  "+n)
