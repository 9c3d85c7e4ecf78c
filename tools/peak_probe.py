import sys, torch
sys.path.insert(0, '.')
import bench
print(bench.measure_peaks(torch.device('cuda:0')))
