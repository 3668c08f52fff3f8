# A/B of an environment knob on the C3 step and the producer+resolve alone: VAR=name VALS="a b"
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for v in $VALS; do
  echo "$VAR=$v $(env $VAR=$v timeout -k 10 120 python -u tools/drawsbench.py 4096 | tail -1) $(env $VAR=$v timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done; done
