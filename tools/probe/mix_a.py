import sys; sys.path.insert(0,'/root/repo')
import torch
print("torch sees", torch.cuda.device_count(), torch.cuda.is_available())
x = torch.ones(4, device='cuda:0'); print("torch alloc ok", x.sum().item())
import jsraytracer_amd as jr
from oracle import pyoracle
sc = jr.Scene(pyoracle.golden_scene('ASimpleScene'))
rgba, col, st = sc.render(32, 32, 1, 4, 1, 1)
print("jsrt ok", rgba.sum(), st)
y = torch.zeros(8, dtype=torch.int32, device='cuda:0')
print("torch again ok", y.sum().item())
