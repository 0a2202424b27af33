set -x
env | grep -i -E "HIP|ROCR|CUDA|GPU" | grep -v GRAFT
timeout -k 5 60 python -c "
import torch; print(torch.cuda.is_available(), torch.cuda.device_count())
x=torch.zeros(1,device='cuda'); print(x)
import sys; sys.path.insert(0,'.')
from adam_amd import bqsr
c=bqsr.Context.get(0); print('ctx ok')
"
timeout -k 5 120 python -u -m pytest tests/test_gpu_staged.py -x -q --timeout 60 --timeout-method thread 2>&1 | tail -3
