set -e
for sz in 4096 8192; do for h in 8 0; do
  SIZE=$sz HELPERS=$h TAG="size $sz helpers $h" CHECK=1 timeout -k 10 120 python -u scripts/lone.py
done; done
timeout -k 10 200 python -u scripts/c5_seq.py
