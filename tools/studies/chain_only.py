import sys, torch
sys.path.insert(0, '.')
import bench, superbblas_amd as sb
print(bench.chain_bench(sb, torch.device('cuda:0')))
