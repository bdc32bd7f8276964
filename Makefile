# Builds the gfx950 HIP library behind include/fall3.h and the C oracle pieces.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := fall_multimodal_amd/csrc
BLD := build
FLAGS := -O3 --offload-arch=$(ARCH) -fPIC -std=c++17 -Iinclude -I$(SRC) -Wno-unused-result
OBJS := $(BLD)/gemm.o $(BLD)/gemm_bf16.o $(BLD)/gemm_glds.o $(BLD)/gemm_big.o $(BLD)/gemm_x3.o $(BLD)/tcn64.o $(BLD)/pw_gemm.o $(BLD)/layers.o $(BLD)/layer0.o $(BLD)/rgb.o $(BLD)/sensor.o $(BLD)/head.o $(BLD)/net.o $(BLD)/targcn.o $(BLD)/targcn_net.o $(BLD)/sktr.o $(BLD)/sktr_net.o $(BLD)/musa.o $(BLD)/musa_net.o
LIB := fall_multimodal_amd/libfall3.so
HDRS := $(wildcard $(SRC)/*.h) include/fall3.h

all: $(LIB)

$(BLD):
	mkdir -p $(BLD)

$(BLD)/%.o: $(SRC)/%.hip $(HDRS) | $(BLD)
	$(HIPCC) $(FLAGS) -c $< -o $@

$(BLD)/%.o: $(SRC)/%.cpp $(HDRS) | $(BLD)
	$(HIPCC) $(FLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -fPIC -o $@ $(OBJS)

clean:
	rm -rf $(BLD) $(LIB)

.PHONY: all clean
