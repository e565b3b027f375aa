mkdir -p gpurun_out/r06h
for d in 15 8 4 2 1; do
  FD_VERIFY_SVC_IO_DBG=$d timeout -k 5 30 integration/_build/svc_probe 64 > gpurun_out/r06h/probe_$d.txt 2>&1
  echo "rc=$?" >> gpurun_out/r06h/probe_$d.txt
done
(dmesg 2>&1 | tail -30) > gpurun_out/r06h/dmesg.txt
true
