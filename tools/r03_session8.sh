# Round-3 closing session: fp16-D2 tests, A/B, every GPU test, then the profile pass and bench line.
bash tools/r03_session5.sh; rc=$?
[[ $rc -ge 124 || $rc -eq 134 || $rc -eq 139 ]] && exit $rc
bash tools/r03_session7.sh
