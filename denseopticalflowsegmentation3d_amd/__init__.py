"""MI355X-native dense-optical-flow clustering + 3D lifting."""
