"""Per-kernel register / spill / occupancy table of one HIP source (hipcc -Rpass-analysis).

usage: python tools/resusage.py pointnerf-slam_amd/csrc/mlp16_bwd.hip [extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '-fno-slp-vectorize', '--offload-arch=gfx950',
       '-I/opt/rocm/include', '-x', 'hip', '-c', src, '-o', '/tmp/_resusage.o',
       '-Rpass-analysis=kernel-resource-usage', *sys.argv[2:]]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r'remark:\s+(.*?): (.*?) \[-Rpass', line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == 'Function Name':
        cur = {'name': v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    name = subprocess.run(['c++filt', r['name']], capture_output=True, text=True).stdout.strip()
    print(f"{name[:70]:70s} V{r.get('VGPRs', '?'):>4} A{r.get('AGPRs', '?'):>4} "
          f"spillV {r.get('VGPRs Spill', '?'):>3} occ {r.get('Occupancy [waves/SIMD]', '?')} "
          f"lds {r.get('LDS Size [bytes/block]', '?')}")
