import sys, json, torch
sys.path.insert(0, ".")
from bench import persistent_bench
dev = torch.device("cuda", 0)
r = [persistent_bench(dev, 65536, 4, 1000, 6000 + i)["ms_per_step"] for i in range(3)]
print(json.dumps({"persistent_ms": r}))
