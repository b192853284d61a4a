import sys,re
def norm(path):
    out=[]
    for l in open(path):
        l=l.split(';')[0].rstrip()
        if not l.strip() or l.strip().startswith('.') and not l.strip().startswith('.LBB'): 
            continue
        if '__hip_cuid_' in l: continue
        out.append(l)
    return out
a,b=norm(sys.argv[1]),norm(sys.argv[2])
print(len(a),len(b),'identical' if a==b else 'DIFFER')
if a!=b:
    import difflib
    d=list(difflib.unified_diff(a,b,lineterm='',n=0))
    print(len(d)); print('\n'.join(d[:40]))
