# round 6: the end-to-end GetTOAs lines and C4 with / without the polled read-backs
TESTK= bash tools/ab.sh gtspin "gtps gt c4" "base lib:varlib/libppfit_nospin.so" 2
