"""CPU emulation of mk::spread (prysm_amd/csrc/keccak_dev.hpp): one Keccak
state spread over a 64-lane wave, with the cross-lane primitives it uses
(DPP row_shl/row_shr/row_ror with row masks, v_permlane16/32_swap,
ds_bpermute) modelled lane by lane.  Checks both word forms (bit-interleaved
e/o and lo/hi) against a textbook Keccak-f[1600]; tests/test_spread_layout.py
runs it on the CPU, tools/spread_debug.hip + tools/spread_debug_cmp.py compare
it with the primitives as the GPU executes them."""
import random
M32=0xFFFFFFFF
RHO=[0,1,62,28,27,36,44,6,55,20,3,10,43,25,39,41,45,15,21,8,18,2,61,56,14]
RC=[0x0000000000000001,0x0000000000008082,0x800000000000808A,0x8000000080008000,0x000000000000808B,0x0000000080000001,0x8000000080008081,0x8000000000008009,0x000000000000008A,0x0000000000000088,0x0000000080008009,0x000000008000000A,0x000000008000808B,0x800000000000008B,0x8000000000008089,0x8000000000008003,0x8000000000008002,0x8000000000000080,0x000000000000800A,0x800000008000000A,0x8000000080008081,0x8000000000008080,0x0000000080000001,0x8000000080008008]
def rotl64(v,r): return ((v<<r)|(v>>(64-r)))&((1<<64)-1) if r else v
def keccak_f(A):
    A=list(A)
    for rnd in range(24):
        C=[A[x]^A[x+5]^A[x+10]^A[x+15]^A[x+20] for x in range(5)]
        D=[C[(x+4)%5]^rotl64(C[(x+1)%5],1) for x in range(5)]
        A=[A[i]^D[i%5] for i in range(25)]
        B=[0]*25
        for x in range(5):
            for y in range(5):
                B[y+5*((2*x+3*y)%5)]=rotl64(A[x+5*y],RHO[x+5*y])
        A=[B[i]^((~B[(i%5+1)%5+5*(i//5)])&B[(i%5+2)%5+5*(i//5)]) for i in range(25)]
        A[0]^=RC[rnd]
    return A
def ilv(v,p): 
    r=0
    for j in range(32): r|=((v>>(2*j+p))&1)<<j
    return r
def unilv(e,o):
    v=0
    for j in range(32): v|=((e>>j)&1)<<(2*j)|((o>>j)&1)<<(2*j+1)
    return v
RCE=[ilv(r,0) for r in RC]; RCO=[ilv(r,1) for r in RC]
def rotl32(v,k): k%=32; return ((v<<k)|(v>>(32-k)))&M32 if k else v
def alignbit(a,b,s): return ((((a<<32)|b)>>(s&31))&M32)
G=0xDEADBEEF
def shl(v,n): return [v[i+n] if (i%16)+n<16 else G for i in range(64)]
def shr(v,n): return [v[i-n] if (i%16)-n>=0 else G for i in range(64)]
def ror8_masked(v):  # row_mask 0xB, old 0
    return [v[16*(i//16)+((i%16)-8)%16] if (i//16) in (0,1,3) else 0 for i in range(64)]
def pl16(a,b):
    a2=list(a); b2=list(b)
    for r0 in (0,2):
        for k in range(16):
            a2[16*(r0+1)+k]=b[16*r0+k]; b2[16*r0+k]=a[16*(r0+1)+k]
    return a2,b2
def pl32(a,b):
    a2=list(a); b2=list(b)
    for k in range(32):
        a2[32+k]=b[k]; b2[k]=a[32+k]
    return a2,b2
def consts(L):
    g=(L>>3)&7; q=L&7; x=q%5; y=g if g<4 else 4
    i=x+5*y; r=RHO[i]; m=r>>1
    sh1=(32-m)&31; sh2=(32-(m+(r&1)))&31
    xs=(3*((y+15-3*x)%5))%5; ys=x
    return dict(i=i,sh1=sh1,sh2=sh2,swap=r&1,src=4*(8*ys+xs),wrap=q==0,iota=M32 if i==0 else 0)
CS=[consts(L) for L in range(64)]
def colsum(v):
    t=[v[i]^u for i,u in enumerate(ror8_masked(v))]
    a,b=pl16(t,t); s=[a[i]^b[i] for i in range(64)]
    a,b=pl32(s,s); return [a[i]^b[i] for i in range(64)]
def rnd(e,o,rce,rco):
    ce=colsum(e); co=colsum(o)
    me=[shl(ce,4)[i] if CS[i]['wrap'] else shr(ce,1)[i] for i in range(64)]
    mo=[shl(co,4)[i] if CS[i]['wrap'] else shr(co,1)[i] for i in range(64)]
    s1o=shl(co,1); s1e=shl(ce,1)
    e=[e[i]^me[i]^alignbit(s1o[i],s1o[i],31) for i in range(64)]
    o=[o[i]^mo[i]^s1e[i] for i in range(64)]
    t1=[alignbit(e[i],e[i],CS[i]['sh1']) for i in range(64)]
    t2=[alignbit(o[i],o[i],CS[i]['sh2']) for i in range(64)]
    re=[t2[i] if CS[i]['swap'] else t1[i] for i in range(64)]
    ro=[t1[i] if CS[i]['swap'] else t2[i] for i in range(64)]
    be=[re[CS[i]['src']//4] for i in range(64)]
    bo=[ro[CS[i]['src']//4] for i in range(64)]
    b1=shl(be,1); b2=shl(be,2); c1=shl(bo,1); c2=shl(bo,2)
    e=[(be[i]^((~b1[i])&b2[i]&M32))^(CS[i]['iota']&rce) for i in range(64)]
    o=[(bo[i]^((~c1[i])&c2[i]&M32))^(CS[i]['iota']&rco) for i in range(64)]
    return e,o


def run_ilv(A):
    e = [ilv(A[c['i']], 0) for c in CS]
    o = [ilv(A[c['i']], 1) for c in CS]
    for r in range(24):
        e, o = rnd(e, o, RCE[r], RCO[r])
    return [unilv(e[8 * (i // 5) + i % 5], o[8 * (i // 5) + i % 5]) for i in range(25)]


def rnd_lh(lo,hi,rcl,rch):
    cl=colsum(lo); ch=colsum(hi)
    ml=[shl(cl,4)[i] if CS[i]['wrap'] else shr(cl,1)[i] for i in range(64)]
    mh=[shl(ch,4)[i] if CS[i]['wrap'] else shr(ch,1)[i] for i in range(64)]
    pl=shl(cl,1); ph=shl(ch,1)
    lo=[lo[i]^ml[i]^alignbit(pl[i],ph[i],31) for i in range(64)]
    hi=[hi[i]^mh[i]^alignbit(ph[i],pl[i],31) for i in range(64)]
    out_l=[];out_h=[]
    for i in range(64):
        r=RHO[CS[i]['i']]; sw= r>=32 or r==0; sh=(32-(r&31))&31
        a,b=(lo[i],hi[i]) if sw else (hi[i],lo[i])
        out_h.append(alignbit(a,b,sh)); out_l.append(alignbit(b,a,sh))
    bl=[out_l[CS[i]['src']//4] for i in range(64)]; bh=[out_h[CS[i]['src']//4] for i in range(64)]
    b1=shl(bl,1); b2=shl(bl,2); c1=shl(bh,1); c2=shl(bh,2)
    lo=[(bl[i]^((~b1[i])&b2[i]&M32))^(CS[i]['iota']&rcl) for i in range(64)]
    hi=[(bh[i]^((~c1[i])&c2[i]&M32))^(CS[i]['iota']&rch) for i in range(64)]
    return lo,hi


def run_lh(A):
    lo = [A[c['i']] & M32 for c in CS]
    hi = [A[c['i']] >> 32 for c in CS]
    for r in range(24):
        lo, hi = rnd_lh(lo, hi, RC[r] & M32, RC[r] >> 32)
    return [lo[8 * (i // 5) + i % 5] | (hi[8 * (i // 5) + i % 5] << 32) for i in range(25)]


if __name__ == "__main__":
    random.seed(1)
    A = [random.getrandbits(64) for _ in range(25)]
    ref = keccak_f(A)
    print("match", run_ilv(A) == ref)
    print("match_lh", run_lh(A) == ref)
