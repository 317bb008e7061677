# debug of the fp8 attention kernel on structured inputs (not a test)
import sys, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/vit-project_amd')
from oracle import attn_fp8_ref as F8
from vit_amd import ops
def run(q,k,v,scale=None):
    B,H,N,_=q.shape; D=H*64
    pack=lambda t: t.permute(0,2,1,3).reshape(B*N,D)
    qkv=torch.cat([pack(q),pack(k),pack(v)],1).to(torch.bfloat16).cuda()
    o,lse=ops.sdpa_fwd(qkv,B,H,N,scale=scale,fp8=True); torch.cuda.synchronize()
    got=o.float().cpu().reshape(B,N,H,64).permute(0,2,1,3)
    ref,rl=F8.sdpa_fp8(q,k,v,scale=scale)
    return got[0,0],ref[0,0]
N=32
eye=torch.zeros(1,1,N,64)
for i in range(N): eye[0,0,i,i]=1
v=eye.clone()
for half in (0,1):
    k=torch.zeros(1,1,N,64); q=torch.zeros(1,1,N,64)
    for i in range(N): k[0,0,i,i+32*half]=1; q[0,0,i,i+32*half]=8
    g,r=run(q,k,v,scale=1.0)
    print('half',half,'argmax got',g[:, :32].argmax(-1).tolist())
    print('        ref',r[:, :32].argmax(-1).tolist())
# diagonal S with value pattern: S[q][key] = q-dependent on key = (q+3)%32
k=torch.zeros(1,1,N,64); q=torch.zeros(1,1,N,64)
for i in range(N): k[0,0,i,i]=1
for i in range(N): q[0,0,i,(i+3)%N]=8
g,r=run(q,k,v,scale=1.0)
print('shift3 got',g[:, :32].argmax(-1).tolist())
print('shift3 ref',r[:, :32].argmax(-1).tolist())
