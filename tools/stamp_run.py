import os, numpy as np, sys
os.environ["MGP_LIBRARY"]="var/stamp/libmgpoisson.so"; os.environ["MGP_STAMP_R"]="1"; os.environ["MGP_GRAPH"]="0"
sys.path.insert(0,"lua-multigrid-poisson_amd")
import mgpoisson
ctx=mgpoisson.Context(mgpoisson.make_opts(dim=3,n=(512,512,512),real="float",smoother="rbgs",nu1=2,nu2=2,prolong="linear"))
ctx.init_point_charge()
for _ in range(3): ctx.cycle()
lex=ctx.get_f(1)  # (z, y, x) lexicographic; raw packed index q of plane 0, colour 0: row j = q // 128, x = 2 (q % 128) + (j & 1)
q=np.arange(256*64); j=q//128; x=2*(q%128)+(j&1)
f=lex[0, j, x].view(np.uint32).astype(np.uint64)
st=(f[0::2] | (f[1::2] << np.uint64(32))).reshape(256,32).astype(np.int64)
np.save("gpurun_out/stamps.npy", st)
print("saved", st[:2,:4])
