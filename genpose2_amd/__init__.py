"""GenPose++ pose-candidate path, MI355X-native."""
