set -o pipefail
mkdir -p gpurun_out/r5
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --cpu-seconds 0 > gpurun_out/r5/ab_timer_on_$i.json 2>>gpurun_out/r5/ab_timer.err || exit $?
  timeout -k 10 200 python3 bench.py --cpu-seconds 0 --no-trial-timer > gpurun_out/r5/ab_timer_off_$i.json 2>>gpurun_out/r5/ab_timer.err || exit $?
done
