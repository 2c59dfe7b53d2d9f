import itertools
G=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G=G+[[l+32 for l in g] for g in G]
RS=272; ZROW=256
def build(order_C, order_A, order_D, order_B, order_E):
    rows=[None]*256
    # A: x=0 cells
    A=[(b,0,y) for b in range(6) for y in range(1,5)]
    A=sorted(A,key=order_A)+[(b,0,0) for b in range(4)]+[(b,0,5) for b in range(4)]
    B=sorted([(b,x,0) for b in range(6) for x in range(1,6)],key=order_B)+[(4,0,0),(5,0,0)]
    C=sorted([(b,x,y) for b in range(6) for x in range(1,6) for y in range(1,5)],key=order_C)+[(4,0,5),(5,0,5),(4,6,0),(5,6,0),(4,6,5),(5,6,5),(5,4,5),(5,5,5)]
    D=sorted([(b,6,y) for b in range(6) for y in range(1,5)],key=order_D)+[(b,6,0) for b in range(4)]+[(b,6,5) for b in range(4)]
    E=sorted([(b,x,5) for b in range(5) for x in range(1,6)]+[(5,1,5),(5,2,5),(5,3,5)],key=order_E)
    allc=A+B+C+D+E
    assert len(allc)==252 and len(set(allc))==252
    for i,c in enumerate(allc): rows[i]=c
    inv={c:i for i,c in enumerate(allc)}
    return rows,inv
def cost(rows,inv,zsel):
    tot=0;n=0
    for T in range(8):
        for tap in range(9):
            dx,dy=tap//3-1,tap%3-1
            rr=[rows[r] for r in range(T*32,T*32+32)]
            if not any(c and 0<=c[1]+dx<7 and 0<=c[2]+dy<6 for c in rr): continue
            for kk in range(8):
                for g in G:
                    banks={}
                    for l in g:
                        r=T*32+(l&31); h=l>>5; c=rows[r]
                        if c and 0<=c[1]+dx<7 and 0<=c[2]+dy<6: nr=inv[(c[0],c[1]+dx,c[2]+dy)]
                        else: nr=ZROW+zsel(r,tap)
                        a=nr*RS+kk*32+16*h
                        for k in range(4):
                            banks.setdefault(((a//4)+k)%64,set()).add(a//4+k)
                    tot+=max(len(s) for s in banks.values()); n+=1
    return tot/n
