"""Host simulation of the packet traversal's node step (trace.hip pkt_nodes): the branchy step
(0-based wave stack) against the branch-free form measured in r5zv (1-based stack with kSentinel at
entry 0, push / pop / next node by selects), on random binary trees with per-lane hit masks and box
distances.  Prints "equal" when both visit the same node / leaf sequence on every tree.
usage: python tools/pkt_step_sim.py"""
import random
S=0x7fffffff
def run(tree, hitf, root, new):
    st=[None]*64; sp=0; node=root; seq=[]
    if new: st[0]=S
    while True:
        while 0<=node<S:
            top = st[sp] if new else None
            seq.append(node)
            dx,dy=tree[node]; h0,h1,t0,t1=hitf[node]   # per-lane lists
            b0=any(h0); b1=any(h1)
            near0=sum(1 for a,b,x,y in zip(h0,h1,t0,t1) if a and b and x<=y); both=sum(1 for a,b in zip(h0,h1) if a and b)
            if not new:
                if not b0 and not b1:
                    if sp>0: sp-=1; node=st[sp]
                    else: node=S
                elif b0 and b1:
                    f=2*near0>=both; st[sp]=dy if f else dx; sp+=1; node=dx if f else dy
                else: node=dx if b0 else dy
            else:
                a0=int(b0); a1=int(b1); two=a0&a1
                f=a0 & int(2*near0>=both)
                st[sp+1]=dy if f else dx
                node=(dx if f else dy) if (a0|a1) else top
                sp+=two-(1-(a0|a1))
        if node==S: break
        seq.append(('leaf',node))
        if new: node=st[sp]; sp-= 1 if sp>0 else 0
        else:
            if sp>0: sp-=1; node=st[sp]
            else: node=S
    return seq
random.seed(2)
for trial in range(20000):
    n=random.randint(1,30); tree={}; nxt=[1]; lc=[-1]
    def build(i,d):
        ch=[]
        for _ in range(2):
            if nxt[0]<n and d<20 and random.random()<0.6: c=nxt[0]; nxt[0]+=1; ch.append(c)
            else: ch.append(lc[0]); lc[0]-=1
        tree[i]=tuple(ch)
        for c in ch:
            if c>=0: build(c,d+1)
    build(0,0)
    L=4
    hitf={i:([random.random()<0.4 for _ in range(L)],[random.random()<0.4 for _ in range(L)],[random.random() for _ in range(L)],[random.random() for _ in range(L)]) for i in tree}
    assert run(tree,hitf,0,False)==run(tree,hitf,0,True), trial
print("equal")
