cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then export FZ_LIB_PATH=""; else export FZ_LIB_PATH=$PWD/tse-replication-package-1-million-fuzzing-sessions_amd/csrc/build/variants/libfz_$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab_$v -o p -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --probe-steps 0 > gpurun_out/pab_$v.log 2>&1 || exit $?
done
