import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
print("torch avail", torch.cuda.is_available(), flush=True)
x = torch.arange(10, device="cuda")
import importlib
DG = importlib.import_module("incubator-druid_amd.datagen")
Q = importlib.import_module("incubator-druid_amd.query")
R = importlib.import_module("incubator-druid_amd.runners")
S = importlib.import_module("incubator-druid_amd.segment")
p = DG.write_basic_segment("/tmp/probe_seg", 50_000, seed=1)
seg = S.GpuSegment(p)
q = Q.GroupByQuery(intervals=["1970-01-01/2020-01-01"], dimensions=["dimZipf"], aggregations=[Q.count("rows")])
res = R.groupby_run([seg], q)
print("groups", res.groups, flush=True)
print("torch still", torch.cuda.is_available(), x.sum().item(), flush=True)
