"""MI355X-native drop-in for ThorLL/Element-Crush-Gym's ``match3tile`` package.

    from match3tile.env import Match3Env            # gym-style single board
    from match3tile.boardv2 import BoardV2           # mctslib State
    from match3tile.boardConfig import BoardConfig
    from match3tile.batched import BatchedMatch3Env  # n boards per GPU

Put ``element-crush-gym_amd/`` on sys.path. All rule evaluation runs in the
HIP kernels of ``element-crush-gym_amd/build/libm3.so``; there is no CPU path.
"""
