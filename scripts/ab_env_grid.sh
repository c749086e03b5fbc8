set -o pipefail
for i in 1 2; do
  for v in 0 1; do echo -n "RT_LDS_GRID=$v: "; RT_LDS_GRID=$v timeout -k 10 120 python scripts/probe_speed.py rtow 256 f64,f32 | tr '\n' ' '; echo; done
done
