"""select_best_gpu (auto_select_gpu.py:3-46 in the reference polls NVML). On an MI355X node each process
owns one GPU: the rank's LOCAL_RANK (one process per GPU, torch.distributed over RCCL)."""
import os


def select_best_gpu(min_free_memory: float = 35.0) -> int:
    return int(os.environ.get('LOCAL_RANK', 0))
