# round 6: streaming (nontemporal) loads/stores everywhere (default build)
# against the first A/B's winner (k_xspec_w2 + k_pass only)
TESTK=all bash tools/ab.sh nta "c2 c3 c5" "base lib:varlib/libppfit_nt3only.so" 2 && \
bash tools/ab.sh ntb "c4 nb1000 nb1023" "base lib:varlib/libppfit_nt3only.so" 1
