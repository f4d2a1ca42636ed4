# Per-workgroup stamps of the resident kernel (TSG_RES_DUMP=2 stderr) by XCD, and the end deviation vs match count.
# Usage: python3 tools/res_stamps_ana.py <dump.err> ...
import sys, numpy as np
for f in sys.argv[1:]:
    xs=[];runs=[];seen=[];ends=[];cnts=[]
    for ln in open(f):
        if ln.startswith("[tsg] resident xsplit:"): xs.append([float(x) for x in ln.split(":")[1].split()])
        elif ln.startswith("[tsg] resident runs:"): runs.append([int(x) for x in ln.split(":")[1].split()])
        elif ln.startswith("[tsg] resident seen:"): seen.append([int(x) for x in ln.split(":")[1].split()])
        elif ln.startswith("[tsg] resident ends:"): ends.append([int(x) for x in ln.split(":")[1].split()])
        elif ln.startswith("[tsg] resident counts:"): cnts.append([int(x) for x in ln.split(":")[1].split()])
    E=np.array(ends[-40:],float)/100; S=np.array(seen[-40:],float)/100; R=np.array(runs[-40:],float); C=np.array(cnts[-40:],float)
    print(f, "n", len(ends), "xf last", np.round(xs[-1],4) if xs else None)
    print(" span mean %.2f  end mean %.2f  end max-mean %.2f" % (E.max(1).mean(), E.mean(), (E.max(1)-E.mean(1)).mean()))
    W=E.shape[1]
    for x in range(8):
        idx=np.arange(x,W,8)
        print("  xcd %d: end mean %.2f  max %.2f  seen %.2f  run %.1f  dur/unit %.4f cnt %.1f" % (x, E[:,idx].mean(), E[:,idx].max(1).mean(), S[:,idx].mean(), R[:,idx].mean(), ((E-S)[:,idx]/R[:,idx]).mean(), C[:,idx].mean()))
    # worst workgroups
    dev=E.mean(0)-E.mean()
    order=np.argsort(dev)[::-1][:12]
    print("  slowest wg:", [(int(w), round(float(dev[w]),2), int(R[0,w]), round(float(C[:,w].mean()),1)) for w in order])

def regress(f):
    ends=[];cnts=[];seen=[]
    for ln in open(f):
        if ln.startswith("[tsg] resident ends:"): ends.append([int(x) for x in ln.split(":")[1].split()])
        elif ln.startswith("[tsg] resident counts:"): cnts.append([int(x) for x in ln.split(":")[1].split()])
        elif ln.startswith("[tsg] resident seen:"): seen.append([int(x) for x in ln.split(":")[1].split()])
    E=np.array(ends[-40:],float)/100; C=np.array(cnts[-40:],float); S=np.array(seen[-40:],float)/100
    dev=(E-E.mean(1,keepdims=True)).mean(0); c=C.mean(0)
    A=np.vstack([np.ones_like(c),c, (np.arange(len(c))%8>=4)]).T
    coef,res,_,_=np.linalg.lstsq(A,dev,rcond=None)
    pred=A@coef
    print(f, "dev = %.3f + %.3f*count + %.3f*[xcd>=4]; resid std %.3f, dev std %.3f" % (coef[0],coef[1],coef[2],(dev-pred).std(),dev.std()))
    for k in range(0,8): print("  count %d: n %d mean dev %.2f" % (k, (np.round(c)==k).sum(), dev[np.round(c)==k].mean() if (np.round(c)==k).any() else float('nan')))
import sys
for f in sys.argv[1:]: regress(f)
