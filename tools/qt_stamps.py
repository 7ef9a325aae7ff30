import sys, os, numpy as np
sys.path.insert(0,'.')
from tests.conftest import load_package
pkg=load_package()
from orbslam3_amd import synth
import torch
fr=synth.frame_batch(64,640,480,seed0=100)
ex=pkg.ORBextractor(1000,1.2,8,20,7,640,480,64)
imgs=torch.from_numpy(fr).cuda()
for _ in range(3): ex.extract_batch_device(imgs,(0,1000))
torch.cuda.synchronize()
NS=12
buf=np.zeros(64*8*NS,np.uint64)
n=ex._lib.orb_debug_qt_stamps(ex._h, buf.ctypes.data, len(buf))
st=buf.reshape(64,8,NS).astype(np.float64)
st[:,:,8]=(buf.reshape(64,8,NS)[:,:,8] & 0xffff).astype(np.float64)
import os
names=["gather","roots","r_node","r_key","sort","c_node","c_key","final","np0","#reg","#car","K"]
for l in range(8):
    m=st[:,l,:].mean(axis=0); mx=st[:,l,:].max(axis=0)
    print(l, " ".join(f"{nm}={m[i]:.0f}/{mx[i]:.0f}" for i,nm in enumerate(names)))
