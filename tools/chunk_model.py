"""Fluid model of run_host's two-stream chunk pipeline (csrc/capi.hip ChunkPlan), used to choose the
chunk plan: the host thread copies chunk j in (blocking), launches it, then waits for chunk j - 1's
kernel and copies its output out; kernels in flight share the GPU equally and last at least one
block lifetime. Copies at the 56 GB/s the r06w trace shows for pageable 33 MB pieces.
    python3 tools/chunk_model.py
Calibration: 2^25 G1 points with the ramp plan, model 0.86 % over device-resident, measured
0.6-1.6 % (profiles/r06x_ab_host_api); the equal-chunk plan, model 1.8 %, measured 2.0-2.3 %."""
# Fluid model of run_host with two streams: in-flight kernels share the GPU equally; the host loop
# is H2D(j) (blocking), launch(j), drain(j-1) (wait kernel j-1, then D2H blocking).
def simulate(sizes, ns=16.0, rin=48, rout=96, bw=56e9, L=2.1e6):
    # returns total time (ns); kernels: remaining work in ns of full-GPU time; min duration L (one block lifetime)
    t=0.0; active={}  # j -> [remaining_work, start_time]
    done={}
    def advance(until):
        nonlocal t
        while active and t < until:
            k=len(active); rem=min(v[0] for v in active.values())
            dt=rem*k
            if t+dt<=until:
                t+=dt
                for j in list(active):
                    active[j][0]-=rem
                    if active[j][0]<=1e-9:
                        # a kernel lasts at least one block lifetime
                        done[j]=max(t, active[j][1]+L); del active[j]
            else:
                step=(until-t)/k
                for j in active: active[j][0]-=step
                t=until
        t=max(t,until)
    def wait_kernel(j):
        while j not in done:
            advance(t+1e5 if active else t)
            if not active and j not in done: raise RuntimeError
        return done[j]
    for j,m in enumerate(sizes):
        advance(t+m*rin/bw*1e9)           # H2D(j) (host busy, GPU keeps running)
        active[j]=[m*ns, t]               # launch
        if j>0:
            e=wait_kernel(j-1); advance(max(t,e)); advance(t+sizes[j-1]*rout/bw*1e9)
    e=wait_kernel(len(sizes)-1); advance(max(t,e)); advance(t+sizes[-1]*rout/bw*1e9)
    return t/1e6
def plan(n, up=4, down=0.5, s0=1<<17, se=1<<17):
    cmax=min(n,1<<21)
    if n>(2<<17): cmax=min(cmax,max(1<<17,((n+7)//8+255)&~255))
    ups=[]; x=s0
    while x<cmax: ups.append(x); x*=up
    downs=[]
    if down:
        x=int(cmax*down)//256*256
        while x>=se: downs.append(x); x=int(x*down)//256*256
        if downs and downs[-1]!=se: downs.append(se)
    rest=n-sum(ups)-sum(downs); mid=[]
    while rest>0: mid.append(min(cmax,rest)); rest-=mid[-1]
    return ups+mid+downs
def old(n):
    chunk=min(n,1<<21)
    if n>(2<<17): chunk=min(chunk,max(1<<17,((n+7)//8+255)&~255))
    s=[]; r=n
    while r>0: s.append(min(chunk,r)); r-=s[-1]
    return s
for n,ns,rin,rout,L,nm in ((1<<25,16.0,48,96,2.1e6,"G1 2^25"),(1<<23,16.0,48,96,2.1e6,"G1 2^23"),(1<<20,25.9,96,192,3.4e6,"G2 2^20"),(1<<21,25.9,96,192,3.4e6,"G2 2^21")):
    dev=n*ns/1e6
    for lab,s in (("old",old(n)),("ramp .5",plan(n)),("ramp .7",plan(n,down=0.7)),("ramp .8",plan(n,down=0.8)),("up only",plan(n,down=0))):
        T=simulate(s,ns,rin,rout,L=L)
        print(f"{nm:8s} {lab:8s} chunks {len(s):3d} {T:8.2f} ms dev {dev:7.2f} over {100*(T/dev-1):5.2f}%")
print('-- G2 2^20 variants')
n=1<<20
for lab,s in (("old 2^17x8",old(n)),("2^16x16",[1<<16]*16),("2^16,2^17..,2^16",[1<<16]+[1<<17]*7+[1<<16]),("2^15,2^16,2^17..,2^16,2^15",[1<<15,1<<16]+[1<<17]*7+[1<<15]),("2^18x4",[1<<18]*4)):
    T=simulate(s,25.9,96,192,L=3.4e6); print(f"{lab:28s} {T:7.2f} over {100*(T/(n*25.9/1e6)-1):5.2f}%")
print('-- s0/se 2^16 vs 2^17')
for n,ns,rin,rout,L,nm in ((1<<25,16.0,48,96,2.1e6,"G1 2^25"),(1<<23,16.0,48,96,2.1e6,"G1 2^23"),(1<<21,25.9,96,192,3.4e6,"G2 2^21"),(1<<21,16.0,48,96,2.1e6,"G1 2^21"),(1<<20,16.0,48,96,2.1e6,"G1 2^20"),(1<<19,25.9,96,192,3.4e6,"G2 2^19")):
    dev=n*ns/1e6
    for lab,s in (("s17",plan(n)),("s16",plan(n,s0=1<<16,se=1<<16)),("s16/e17",plan(n,s0=1<<16)),("s17/e16",plan(n,se=1<<16))):
        T=simulate(s,ns,rin,rout,L=L); print(f"{nm:8s} {lab:8s} chunks {len(s):3d} over {100*(T/dev-1):5.2f}%")
