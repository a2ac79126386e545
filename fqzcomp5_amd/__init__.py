"""MI355X-native fqzcomp5 block codec."""
