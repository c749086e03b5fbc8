set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_defer.log
timeout -k 10 200 bash scripts/ab_lib.sh "rtow 256 f64" k1 k8 k16 k24 > $L 2>&1 || exit 1
echo "-- mesh50k" >> $L; timeout -k 10 200 bash scripts/ab_lib.sh "mesh50k 64 f64" k1 k16 >> $L 2>&1 || exit 1
echo "-- cornell" >> $L; timeout -k 10 120 bash scripts/ab_lib.sh "cornell 64 f64" k1 k16 >> $L 2>&1 || exit 1
echo "-- rtow grid global" >> $L; RT_LDS_GRID=0 timeout -k 10 120 bash scripts/ab_lib.sh "rtow 128 f64" k1 k16 >> $L 2>&1 || exit 1
echo "-- rtow f32" >> $L; timeout -k 10 120 bash scripts/ab_lib.sh "rtow 256 f32" k1 k16 >> $L 2>&1 || exit 1
echo "-- progressive k16" >> $L; RT_HIP_LIB=blenderraytracer_amd/lib/variants/k16.so timeout -k 10 100 python -u scripts/probe_progressive.py 5 >> $L 2>&1
