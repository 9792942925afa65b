// Exhaustive check: is there a circuit of three 3-input gates (v_bitop3) for the B3/S23 rule
// given the vertical adder outputs o, co, p, q and the alive bit (gol_kernels.hip life_bits)?
// Prints "found 0": the rule stage needs 4 gates, so 8 v_bitop3 per output word is minimal for
// this adder structure.   gcc -O2 -o /tmp/rs tools/rule_search.c && /tmp/rs
#include <stdio.h>
#include <stdint.h>
int main(){
  // 32 rows: bit i of input var v = (row>>v)&1 ; vars: 0=o 1=co 2=p 3=q 4=alive
  uint32_t in[5]; for(int v=0;v<5;v++){in[v]=0;for(int r=0;r<32;r++) if((r>>v)&1) in[v]|=1u<<r;}
  uint32_t f=0, care=0;
  for(int r=0;r<32;r++){int o=r&1,co=(r>>1)&1,p=(r>>2)&1,q=(r>>3)&1,al=(r>>4)&1;
    int s=o+2*(co+p)+4*q; int nx=(s==3)||(al&&s==4); if(nx) f|=1u<<r; care|=1u<<r;}
  long found=0;
  uint32_t sig[8];
  for(int v=0;v<5;v++) sig[v]=in[v];
  // apply LUT tt to signals x,y,z (tt index = 4a+2b+c with a=x? we use bit (a<<2|b<<1|c))
  #define LUT(tt,x,y,z) ({uint32_t _r=0; for(int _k=0;_k<8;_k++) if((tt>>_k)&1){ uint32_t m=((_k&4)?x:~x)&((_k&2)?y:~y)&((_k&1)?z:~z); _r|=m;} _r;})
  for(int a=0;a<5;a++)for(int b=a+1;b<5;b++)for(int c=b+1;c<5;c++)for(int t1=0;t1<256;t1++){
    sig[5]=LUT(t1,sig[a],sig[b],sig[c]);
    for(int d=0;d<6;d++)for(int e=d+1;e<6;e++)for(int g=e+1;g<6;g++){ // g2 must use g1 (else reorder)
      for(int t2=0;t2<256;t2++){
        sig[6]=LUT(t2,sig[d],sig[e],sig[g]);
        // final gate: 3 signals among 7 must determine f
        for(int x=0;x<7;x++)for(int y=x+1;y<7;y++)for(int z=y+1;z<7;z++){
          uint32_t X=sig[x],Y=sig[y],Z=sig[z]; int ok=1; int tt=0,seen=0;
          for(int k=0;k<8&&ok;k++){uint32_t m=((k&4)?X:~X)&((k&2)?Y:~Y)&((k&1)?Z:~Z)&care; if(!m) continue;
            if((m&f)==m) {tt|=1<<k;} else if((m&f)==0){} else ok=0;}
          if(ok){found++; if(found<=10) printf("g1=%d(%d,%d,%d) g2=%d(%d,%d,%d) g3(%d,%d,%d)\n",t1,a,b,c,t2,d,e,g,x,y,z);}
        }}}
  }
  printf("found %ld\n",found);
  // also 2-gate check happens implicitly if final uses not g2
}
