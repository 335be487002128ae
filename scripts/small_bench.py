"""cfg4 (QAT) and cfg5 (DONN) secondary timings only, for A/B runs of library variants."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
q = bench.bench_qat(dev, 0, 1, steps=200)
d = bench.bench_donn(dev, 0, 1)
print(json.dumps({"qat": {k: v["ms_per_it"] for k, v in q["phases"].items()},
                  "donn": {k: v["ms_per_step"] for k, v in d["modes"].items()}}))
