for o in "locked=1" "locked=0" "locked=2" "locked=1 wpc=16" "locked=1 wpc=8"; do timeout -k 10 120 python tools/c5_profile.py quad $o | tail -1 || exit 1; done
