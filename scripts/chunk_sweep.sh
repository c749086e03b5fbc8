for c in 34 48 64 96 34; do echo -n "c$c "; RT_POOL_CHUNK=$c timeout -k 10 120 python scripts/probe_speed.py rtow 512 f64 | sed -e 's/wall.*kernel,//' -e 's/segments.*//'; done
for c in 12 16 24 32 12; do echo -n "c$c "; RT_POOL_CHUNK=$c timeout -k 10 120 python scripts/probe_speed.py mesh50k 256 f64 | sed -e 's/wall.*kernel,//' -e 's/segments.*//'; done
