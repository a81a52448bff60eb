"""mlic_amd: MI355X-native MLIC++ encode/decode (HIP/CDNA4) behind the CompressAI API."""
