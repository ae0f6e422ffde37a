bash tools/r06_onepass_prof.sh r06g && bash tools/ab/r06_op_probe_run.sh r06g nolb nostore norender tpw2 w1 w2 w1t2 w2t2
