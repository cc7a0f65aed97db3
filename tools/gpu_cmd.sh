export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ab.py --libs old,base,sc1nd,plain --bench "--steps 20" --reps 2 || exit 1
timeout -k 10 300 python tools/ab.py --libs old,base,sc1nd,plain --reps 2 || exit 1
