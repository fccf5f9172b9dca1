set -u
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1
for np in 1 2; do
 for so in 0 force; do
  for pd in 1 128; do
    tmp=$(mktemp /tmp/sp.XXXXXX.json)
    HICCL_DRIVER_JSON=$tmp HICCL_STREAM_ORDERED=$so HICCL_GRAPH=0 timeout -k 10 120 $mpirun -np $np build/collectives_hip_f32 8 $((1<<20)) 1 1 $pd 2 10 $np ipc > /dev/null 2>&1
    python3 -c "import json; r=json.load(open('$tmp')); print(json.dumps(dict(np=$np, so='$so', pd=$pd, med=r['collective_ms_median'], mode=r['mode'], kat=r['kat'], ksteps=r['kernel_steps_rank0'])))"
    rm -f $tmp
  done
 done
done
