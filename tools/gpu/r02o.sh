# r02o: what-if timing builds (critical path of k_dyn4), interleaved A/B
bash tools/gpu/ab.sh r02o base wi_fwd wi_bwd wi_both wi_nohc
