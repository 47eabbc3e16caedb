cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5e}
mkdir -p $O
ITR_HOST_TIMING=1 timeout -k 10 300 python scripts/host_wrap_timing.py 5 > $O/host_wrap.txt 2>&1 || { tail $O/host_wrap.txt; exit 1; }
cat $O/host_wrap.txt
uname -r; nproc; grep -i "model name" /proc/cpuinfo | head -1; cat /sys/kernel/mm/transparent_hugepage/enabled
