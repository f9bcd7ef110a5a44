"""Model zoo: MLP, LeNet-style CNN, AlexNet, ResNet-18/34/50/101/152, BERT."""
