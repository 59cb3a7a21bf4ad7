"""Compare tools/spread_debug (GPU dump of the spread primitives and one
round, gpurun_out/spread_debug.json) with the CPU emulation."""
import json, sys
sys.path.insert(0, 'tools')
from spread_emu import *  # noqa: E402,F401,F403
d=json.load(open('/root/repo/gpurun_out/spread_debug.json'))
v=d['in'][:64]; w=d['in'][64:]; out=[d['out'][64*k:64*k+64] for k in range(22)]
e,o=v,w
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
canon=[i for i in range(64) if (i&7)<5 and (i>>3)<5]
for k,exp,lanes in [(14,me,canon),(15,mo,canon),(16,e,canon),(17,o,canon),(18,re,canon),(19,ro,canon),(20,be,range(64)),(21,bo,range(64))]:
    bad=[i for i in lanes if exp[i]!=out[k][i]]
    print(k,'ok' if not bad else f'bad {bad[:16]} ({len(bad)})')
