bash tools/gpu_session.sh r06c ab:main,main+ARGS=--streams/4608,main+ARGS=--streams/5120,main+SLAM2D_PIPELINE=1 && \
bash tools/gpu_session.sh r06d prof:gm:--config,gmapping bench:karto:--config,karto,--no-cpu-baseline bench:kloop:--config,karto_loop,--no-cpu-baseline
