set -e
timeout -k 10 120 python -u tools/sync_repro.py 2>&1 | grep -v -e Warning -e amdgpu.ids
