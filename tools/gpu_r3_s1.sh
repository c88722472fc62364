set -o pipefail
{ id; ls -l /dev/net/tun; unshare -rn sh -c 'id; cat /proc/self/status | grep Cap; python3 -c "
import os,fcntl,struct
fd=os.open(\"/dev/net/tun\",os.O_RDWR)
fcntl.ioctl(fd,0x400454CA,struct.pack(\"16sH\",b\"tprobe0\",0x1002))
print(\"tap ok\")
"'; echo "userns rc=$?"; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > gpurun_out/r3_s1_env.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_s1_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_s1_bench.json 2> gpurun_out/r3_s1_bench.err
