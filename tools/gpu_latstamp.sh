cd $GRAFT_REPO_ROOT
PTV_STAMP_LATTICE=1 timeout -k 10 200 python tools/quick_time.py 512 5000000 8 --stamps
PTV_STAMP_LATTICE=1 PTV_NO_LAT_ORDER=1 timeout -k 10 200 python tools/quick_time.py 512 5000000 8 --stamps
