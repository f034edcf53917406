"""mpc_ros_amd -- MI355X-native batched NMPC solver for the mpc_ros MPC::Solve hot path."""
