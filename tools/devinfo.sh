python -c "
import torch
p=torch.cuda.get_device_properties(0)
print(p)
print('CUs', p.multi_processor_count, 'mem GiB', p.total_memory/2**30)
"
rocminfo 2>/dev/null | grep -E "Compute Unit|Marketing|SIMDs per CU|Max Clock|Name:.*gfx" | head -12
rocm-smi --showcomputepartition --showmemorypartition 2>/dev/null | head -20
rocm-smi --showclocks 2>/dev/null | head -20
