"""cfg3 CZT calls for a rocprofv3 kernel trace: python3 scripts/czt_prof.py [calls]."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import bench  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    r = bench.bench_czt(torch.device("cuda:0"), 0, 1, steps=calls, warmup=1)
    print(r)


if __name__ == "__main__":
    main()
